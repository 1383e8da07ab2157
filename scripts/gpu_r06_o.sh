# Round 6, fifteenth pass: the resolve's taps requested with the quad's
# corners (key -> corners -> taps becomes key -> corners +
# taps; a position in the claimed quad's triangle lies in [qi, qi+1] x [qj,
# qj+1], so slice 0's taps are the quad's own points unless it sits on the far
# edge).  Arms: spec (3 rows, 5 waves per SIMD: spills), spec4 (3 rows, 4
# waves), spec2r (2 rows per thread, 5 waves), spec2r6 (2 rows, 6 waves), p2r
# (the product with 2 rows: the control for the item shape).
# The rectify suite on each, then interleaved timing and resolve stats.
#   bash scripts/gpu_r06_o.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06o}; mkdir -p $O
ARMS="spec4 spec2r spec2r6 p2r spec"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for interp in nearest bilinear; do
  for pass in 1 2; do
    for arm in product $ARMS; do
      L=xcube-resampling_amd/lib/libxrs.so
      [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
      XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 --interp $interp > $O/t_${arm}_${interp}_$pass.log 2>&1 || exit $?
      echo "$arm $interp $pass $(grep 'ms per' $O/t_${arm}_${interp}_$pass.log)"
    done
  done
done
for arm in product spec4 spec2r spec2r6; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm nearest"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
