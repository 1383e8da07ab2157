# Round 5: K3i without the counter memset, second form (no per-item flag
# load): affine / coarsen GPU tests and the config-3 coarsen timed
# interleaved against the previous kernels (probe/k3old); the claim with
# tile-local float32 forms anchored per lane and row (probe/rectpx5):
# rectify GPU tests on it, then K4 + K5 + K6 fused nearest timed interleaved
# against the product, and both arms' kernel stats.
#   bash scripts/gpu_r05_e.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05e}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_configs_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
XRS_LIBRARY=probe/rectpx5/pkg/lib/libxrs.so timeout -k 10 400 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_rect_rectpx5.log 2>&1; rc=$?
echo rectpx5; tail -2 $O/pytest_rect_rectpx5.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base k3old; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_coarsen.py >> $O/k3_ab.log 2> $O/k3_ab_$arm.err || exit $?
    tail -1 $O/k3_ab.log
  done
done
ARMS="base rectpx5"
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
