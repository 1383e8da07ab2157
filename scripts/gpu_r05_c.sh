# Round 5 combined: GPU tests of the changed paths (affine K2 groups, rectify
# float32 claim window, multidevice, sharding), K2 and rectify A/B against
# the previous kernels (probe/k2old, probe/rectold), K1 band-height arms,
# then the config-3 / config-4 lines (config 4 with its VALU-issue PMC pass).
#   bash scripts/gpu_r05_c.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05c}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_affine_gpu.py tests/test_rectify_gpu.py tests/test_multidevice_gpu.py tests/test_sharding_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base rectold; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 >> $O/rect_ab.log 2> $O/rect_ab_$arm.err || exit $?
    tail -1 $O/rect_ab.log
  done
done
for pass in 1 2; do
  for arm in base k2old; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_affine.py --tag $arm >> $O/k2_ab.jsonl 2> $O/k2_ab_$arm.err || exit $?
    tail -1 $O/k2_ab.jsonl
  done
done
for arm in base rectold; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes tiles
done
timeout -k 10 300 python -u scripts/k1_knob_ab.py --passes 2 --arms base,b16,b24,b40,b48,b64 > $O/k1_band.jsonl 2> $O/k1_band.err || exit $?
cat $O/k1_band.jsonl
timeout -k 10 400 python -u scripts/bench_configs.py --configs 3,4 > $O/configs34.jsonl 2> $O/configs34.err || exit $?
cut -c1-250 $O/configs34.jsonl
