# Round 6: the compacted claim walk taking each 16-row strip in two 8-row
# halves (chalf; gpu_r06_x.sh's 8-row strips ran the 2x finer target 2.166 vs
# 2.237 ms, but need other strip counts on the host) — same offsets, twice the
# work units for the compacted walk only.
#   bash scripts/gpu_r06_ab.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06ab}; mkdir -p $O
ARMS="chalf"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for rd in 2 3 1.5 1; do
  for pass in 1 2 3; do
    for arm in product $ARMS; do
      L=xcube-resampling_amd/lib/libxrs.so
      [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
      XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 10 --res-div $rd > $O/t_${arm}_${rd}_$pass.log 2>&1 || exit $?
      echo "$arm $rd $pass $(grep 'ms per' $O/t_${arm}_${rd}_$pass.log)"
    done
  done
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 --res-div 2 > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm res/2"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
