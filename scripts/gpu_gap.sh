# Bench kernel trace (gap between warm-up and timed steps), then K1 probe arms:
# parity tests on each probe library and the bench A/B.   bash scripts/gpu_gap.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --no-traffic --no-f64 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_prof.json')); print('prof run', d['ms_per_step'], d['roofline']['kernel_ms'], d['clock_GHz'])"
python3 scripts/kstats.py $O/prof/bench_kernel_stats.csv gather
for arm in "$@"; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_sharding_gpu.py tests/test_streaming_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$arm.log 2>&1 || { tail -30 $O/pytest_$arm.log; exit 1; }
  echo "$arm: $(tail -1 $O/pytest_$arm.log)"
done
SKIP_TESTS=1 bash scripts/gpu_suite3.sh $O/ab "$@"
