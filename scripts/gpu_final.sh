# Round-end GPU call: scripts/gpu_round.sh (suite, smoke, bench with its PMC
# traffic passes, band rehearsal, 2-rank gloo bench, rocprof of the bench),
# then every config line and the rectify kernel stats.
#   bash scripts/gpu_final.sh OUTDIR
export TMPDIR=/tmp
OUT=${1:-gpurun_out/final}
bash scripts/gpu_round.sh $OUT; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/bench_configs.py --configs 1,2,2u,3,4 --cpu-seconds 8 > $OUT/configs.jsonl 2> $OUT/configs.err || exit $?
cut -c1-160 $OUT/configs.jsonl
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $OUT/bench_w5.json 2> $OUT/bench_w5.err || exit $?
cut -c1-300 $OUT/bench_w5.json
bash scripts/gpu_rect3.sh $OUT/rect fused || exit $?
exit $rc
