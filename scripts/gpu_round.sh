# One GPU call: parity suite, smoke, bench, rocprof kernel stats of the bench.
# Test failures (pytest exit 1) do not stop the later steps; a crash, abort or
# time limit (any other non-zero status) ends the call there.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r01}
mkdir -p $OUT
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with status $rc"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err
timeout -k 10 400 python -u scripts/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err
cat $OUT/configs.jsonl
exit $rc
