# Round 5, rectify claim with the float32 window setup: the rectify GPU tests
# (config 4 whole swath and the claim-form geometries bit-exact against the C
# oracle), then K4+K5+K6 (fused nearest) timed interleaved against the
# previous tree (probe/rectold), then both arms' kernel stats.
#   bash scripts/gpu_r05_rect.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05rect}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py tests/test_multidevice_gpu.py tests/test_sharding_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base rectold; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 >> $O/ab.log 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.log
  done
done
for arm in base rectold; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
done
for arm in base rectold; do
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes tiles
done
