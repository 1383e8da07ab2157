# Round 6, first GPU pass: the rectify suite (whole config-4 swath bit-exact
# against the C oracle, with the wave-compacted claim walk), the new transform
# threshold test, the stream-synchronising unregister, config 5 on all 400
# tiles; the rectify arms' parity on the config-4 swath and the fused-resolve
# tests; K4+K5+K6 (fused nearest) interleaved against round 5 (probe/r5) and
# the arms, with kernel stats; then the K1 prefetch arms.
#   bash scripts/gpu_r06_a.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06a}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rectify_gpu.py tests/test_transform_gpu.py tests/test_streaming_gpu.py tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_multidevice_gpu.py "tests/test_configs_gpu.py::test_config5_full_size_all_tiles" -m gpu -q -x --durations 5 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -12 $O/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest status $rc"; exit $rc; }
for arm in rpf5 rpf4 k4dpp k4wide; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x -k "config4_full or fused_resolve or k4_ or triangle_keys or filled_claim" --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for pass in 1 2 3; do
  for arm in product r5 rpf5 rpf4 k4dpp k4wide; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 > $O/t_${arm}_$pass.log 2>&1 || exit $?
    echo "$arm $pass $(grep 'ms per' $O/t_${arm}_$pass.log)"
  done
done
for arm in product r5 rpf5 rpf4 k4dpp k4wide; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 20 > $O/ks_$arm.log 2>&1 || exit $?
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes tiles
done
# K3i on a grid off the integral layout: product (K3i stops at
# the overflowing item) against round 5
for pass in 1 2; do
  for arm in product r5; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_coarsen.py --frac >> $O/coarsen_frac.log 2>&1 || exit $?
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_coarsen.py >> $O/coarsen_frac.log 2>&1 || exit $?
    tail -2 $O/coarsen_frac.log
  done
done
# K1: next-item coordinate prefetch arms (probe/k1pf*, 2 / 4 items per block),
# parity of one arm on the reproject suite, then interleaved timing
XRS_LIBRARY=probe/k1pflb/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_k1pflb.log 2>&1; rc=$?
tail -2 $O/pytest_k1pflb.log
[ $rc -eq 0 ] || { echo "k1 arm pytest status $rc"; exit $rc; }
for pass in 1 2 3; do
  for arm in product k1pf k1pflb k1pflb4; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --steps 30 --tag $arm >> $O/k1_ab.jsonl 2> $O/k1_ab_$arm.err || exit $?
    tail -1 $O/k1_ab.jsonl | cut -c1-200
  done
done
