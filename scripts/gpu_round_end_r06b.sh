# Round-6 end check of the final tree (after the claim grid, the 7-wave resolve,
# K4 on the resident grid): the whole GPU suite, smoke, the bench line
# (driver settings, with its PMC traffic passes), the rocprofv3 kernel stats
# of the bench command, the secondary config lines, the band rehearsal, and
# the N > 1 bench path rehearsed on this one GPU (gloo ranks sharing it: the
# launcher-free torchrun path the driver takes, its band split, barrier and
# max-over-ranks timing; the numbers of shared-GPU ranks are not a scaling
# measurement).
#   bash scripts/gpu_round_end_r06b.sh OUTDIR
export TMPDIR=/tmp
OUT=${1:-gpurun_out/end6b}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest ended with status $rc"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --warmup 5 --steps 20 > $OUT/bench_w5.json 2> $OUT/bench_w5.err || exit $?
cut -c1-300 $OUT/bench_w5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-traffic --no-f64 --warmup 5 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit $?
cut -c1-200 $OUT/bench_prof.json
timeout -k 10 900 python -u scripts/bench_configs.py --configs 1,2,2u,3,3f,4,4f --cpu-seconds 6 > $OUT/configs.jsonl 2> $OUT/configs.err || { tail -20 $OUT/configs.err; exit 1; }
cut -c1-160 $OUT/configs.jsonl
timeout -k 10 300 python -u scripts/rehearse_bands.py > $OUT/bands.jsonl 2> $OUT/bands.err || exit $?
cut -c1-200 $OUT/bands.jsonl
for n in 2 4; do
  XRS_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --warmup 3 --steps 5 --no-cpu-baseline --no-f64 > $OUT/bench_gloo$n.json 2> $OUT/bench_gloo$n.err || exit $?
  cut -c1-300 $OUT/bench_gloo$n.json
done
