# Round-end check of the tree: GPU suite, smoke, bench (driver settings, with
# its PMC traffic passes), the rocprofv3 kernel stats of the bench command,
# config-4 rectify kernel stats, the secondary config lines with their CPU
# baselines, and the one-GPU rehearsal of the multi-GPU band split.
#   bash scripts/gpu_round_end.sh OUTDIR
export TMPDIR=/tmp
OUT=${1:-gpurun_out/end}
mkdir -p $OUT
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest ended with status $rc"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 1 --warmup 5 --steps 20 > $OUT/bench_w5.json 2> $OUT/bench_w5.err || exit $?
cut -c1-300 $OUT/bench_w5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-traffic --no-f64 --warmup 5 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit $?
cut -c1-200 $OUT/bench_prof.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rect -o c4 -- python3 scripts/time_rectify.py --reps 10 --fused > $OUT/rect_time.log 2>&1 || exit $?
grep "ms per" $OUT/rect_time.log
# the config lines and the band rehearsal: scripts/gpu_round_end2.sh
