# Round 6: K6 (the other variables' sampling, rectify_var_kernel) on 8192 /
# one-pixel-per-thread blocks instead of 2048 (k6g32, k6g1), timed in the
# unfused pass (ij image + K6).
#   bash scripts/gpu_r06_aa.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06aa}; mkdir -p $O
ARMS="k6g32 k6g1"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for interp in nearest bilinear; do
  for pass in 1 2 3; do
    for arm in product $ARMS; do
      L=xcube-resampling_amd/lib/libxrs.so
      [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
      XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --reps 20 --interp $interp > $O/t_${arm}_${interp}_$pass.log 2>&1 || exit $?
      echo "$arm $interp $pass $(grep 'ms per' $O/t_${arm}_${interp}_$pass.log)"
    done
  done
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --reps 10 --interp bilinear > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm bilinear unfused"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) rectify_var resolve claim
done
