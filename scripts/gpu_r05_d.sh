# Round 5: affine / coarsen GPU tests (K3i without the counter memset), the
# config-3 coarsen timed interleaved against the previous kernels
# (probe/k3old), then the K4 arms at config 4 (4 waves per SIMD by launch
# bounds: k4lb4; one 64x16 block per wave: k4grid; both: k4both) and the
# claim with tile-local float32 forms (rectpx3: packed bound, rectpx4:
# unpacked bound; rectify GPU tests first) timed interleaved (K4 + K5 + K6
# fused nearest) with their kernel stats.
#   bash scripts/gpu_r05_d.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05d}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_configs_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
for arm in rectpx4 rectpx3; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 400 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_rect_$arm.log 2>&1; rc=$?
  echo $arm; tail -2 $O/pytest_rect_$arm.log
  case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
done
for pass in 1 2 3; do
  for arm in base k3old; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_coarsen.py >> $O/k3_ab.log 2> $O/k3_ab_$arm.err || exit $?
    tail -1 $O/k3_ab.log
  done
done
ARMS="base k4lb4 k4grid k4both rectpx3 rectpx4"
for pass in 1 2 3; do
  for arm in $ARMS; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 >> $O/k4_ab.log 2> $O/k4_ab_$arm.err || exit $?
    tail -1 $O/k4_ab.log
  done
done
for arm in $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
