# Round 6, ninth pass: resolve arms that load only the picked triangle's three
# corners (6 loads instead of 8; 85 VGPRs at 5 waves per SIMD, or 80 at 6 by
# launch bounds): the rectify suite on each, interleaved config-4 timing and
# kernel stats.   bash scripts/gpu_r06_i.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06i}; mkdir -p $O
ARMS="tri3 tri3lb6"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for pass in 1 2 3; do
  for arm in product $ARMS; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 > $O/t_${arm}_$pass.log 2>&1 || exit $?
    echo "$arm $pass $(grep 'ms per' $O/t_${arm}_$pass.log)"
  done
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 20 > $O/ks_$arm.log 2>&1 || exit $?
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) resolve
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --interp bilinear --reps 20 > $O/tb_${arm}.log 2>&1 || exit $?
  echo "$arm bilinear $(grep 'ms per' $O/tb_${arm}.log)"
done
