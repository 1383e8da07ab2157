# Round 6: the resolve's items dealt to the XCDs in groups of 4 / 8 / 16
# consecutive items (rxg4, rxg8, rxg16: 128-column segments of one 8-row band
# in one L2) at the final occupancy (2 rows, 7 waves, 16384 blocks); round 6's
# first try (3 rows, 5 waves) read less and ran slower (r06c).
#   bash scripts/gpu_r06_ac.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06ac}; mkdir -p $O
ARMS="rxg4 rxg8 rxg16"
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
      XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 --interp $interp > $O/t_${arm}_${interp}_$pass.log 2>&1 || exit $?
      echo "$arm $interp $pass $(grep 'ms per' $O/t_${arm}_${interp}_$pass.log)"
    done
  done
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm nearest"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done

