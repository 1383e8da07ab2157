# Round 5: the resolve loading only the three corners of the triangle the
# claim picked (probe/res3; res3r4: 4 rows per item, res3lb6: 6 waves per
# SIMD): rectify GPU tests on res3, then
# K4 + K5 + K6 fused nearest at config 4 timed interleaved with the product,
# and both arms' kernel stats.
#   bash scripts/gpu_r05_l.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05l}; mkdir -p $O
XRS_LIBRARY=probe/res3/pkg/lib/libxrs.so timeout -k 10 400 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_rect_res3.log 2>&1; rc=$?
echo res3; tail -2 $O/pytest_rect_res3.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
ARMS="base res3 res3r4 res3lb6"
for pass in 1 2 3; do
  for arm in $ARMS; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 >> $O/rect_ab.log 2> $O/rect_ab_$arm.err || exit $?
    tail -1 $O/rect_ab.log
  done
done
for arm in $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
