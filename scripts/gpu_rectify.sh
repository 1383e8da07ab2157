# Rectify iteration call: GPU parity tests of K4/K5/K6, then config 4 timed
# and its rocprofv3 kernel stats.   bash scripts/gpu_rectify.sh [outdir]
export TMPDIR=/tmp
OUT=${1:-gpurun_out/rect}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py tests/test_spatial_gpu.py -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/bench_configs.py --configs 4 --cpu-seconds 1 > $OUT/c4.jsonl 2> $OUT/c4.err || exit $?
cut -c1-400 $OUT/c4.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 scripts/bench_configs.py --configs 4 --cpu-seconds 0.1 > $OUT/c4_prof.log 2>&1 || exit $?
cat $OUT/prof/c4_kernel_stats.csv | cut -c1-200
