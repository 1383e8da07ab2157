# Round-end, second half: the secondary config lines (CPU baselines on the
# whole configs 3 and 4) and the one-GPU rehearsal of the multi-GPU split.
#   bash scripts/gpu_round_end2.sh OUTDIR
export TMPDIR=/tmp
OUT=${1:-gpurun_out/end}
mkdir -p $OUT
timeout -k 10 700 python -u scripts/bench_configs.py --configs 1,2,2u,3,4 --cpu-seconds 6 > $OUT/configs.jsonl 2> $OUT/configs.err || { tail -20 $OUT/configs.err; exit 1; }
cut -c1-160 $OUT/configs.jsonl
timeout -k 10 300 python -u scripts/rehearse_bands.py > $OUT/bands.jsonl 2> $OUT/bands.err || exit $?
cut -c1-200 $OUT/bands.jsonl
