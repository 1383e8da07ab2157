export TMPDIR=/tmp
OUT=${1:-gpurun_out/bench}
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
timeout -k 10 300 python -u scripts/rehearse_bands.py > $OUT/bands.jsonl 2> $OUT/bands.err || exit $?
cut -c1-200 $OUT/bands.jsonl
XRS_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err || exit $?
cat $OUT/bench_2rank_gloo.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-traffic --no-f64 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit $?
