# Rectify suite (dataset fusion for every interpolation), K4 grid arms, config-4 line.
export TMPDIR=/tmp
OUT=gpurun_out/k4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py tests/test_spatial_gpu.py tests/test_sharding_gpu.py tests/test_streaming_gpu.py -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for pass in 1 2; do
  for arm in product kb4 kb16; do
    if [ $arm = product ]; then L=""; else L=$PWD/probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_rectify.py --reps 20 --fused >> $OUT/ab.log 2>&1 || exit $?
  done
done
grep "ms per" $OUT/ab.log
timeout -k 10 600 python -u scripts/bench_configs.py --configs 4 --cpu-seconds 4 > $OUT/configs4.jsonl 2> $OUT/configs4.err || exit $?
cut -c1-120 $OUT/configs4.jsonl
