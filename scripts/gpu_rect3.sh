# Rectify (config 4) A/B: rectify GPU tests on the product library, then
# time_rectify.py under rocprofv3 --kernel-trace --stats for product and arms.
#   bash scripts/gpu_rect3.sh OUTDIR ARM...   (arm "fused": product library, --fused)
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py tests/test_streaming_gpu.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for pass in 1 2; do
  for arm in base "$@"; do
    X=""
    if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so
    elif [ $arm = fused ]; then L=xcube-resampling_amd/lib/libxrs.so; X=--fused
    else L=probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${arm}_$pass -o c4 -- python3 scripts/time_rectify.py --reps 20 $X > $O/${arm}_$pass.log 2>&1 || exit 1
    grep "ms per" $O/${arm}_$pass.log
    python3 scripts/kstats.py $O/${arm}_$pass/c4_kernel_stats.csv bboxes claim resolve rectify_var tiles
  done
done
