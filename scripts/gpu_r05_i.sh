# Round 5: K1 in 1024 x 16 items (product) — reproject-path GPU tests, then
# timed interleaved with the previous commit (probe/k1head); the claim's
# strip-row prefetch — two rows ahead instead of one
# (pf2: 4 waves per SIMD, 3 VGPRs spilled; pf2lb3: 3 waves per SIMD, no
# spill) and 3 waves per SIMD alone (lb3): rectify GPU tests on pf2lb3, then
# K4 + K5 + K6 fused nearest at config 4 timed interleaved with the product,
# and the kernel stats of every arm; last the bench line.
#   bash scripts/gpu_r05_i.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05i}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_sharding_gpu.py tests/test_integration_gpu.py tests/test_streaming_gpu.py tests/test_spatial_gpu.py tests/test_multidevice_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base k1head; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/k1_ab.jsonl 2> $O/k1_ab_$arm.err || exit $?
    tail -1 $O/k1_ab.jsonl
  done
done
XRS_LIBRARY=probe/pf2lb3/pkg/lib/libxrs.so timeout -k 10 400 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_rect_pf2lb3.log 2>&1; rc=$?
echo pf2lb3; tail -2 $O/pytest_rect_pf2lb3.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
ARMS="base pf2lb3 pf2 lb3"
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
timeout -k 10 600 python -u bench.py --gpus 1 --warmup 5 --steps 20 > $O/bench_w5.json 2> $O/bench_w5.err || exit $?
cut -c1-400 $O/bench_w5.json
