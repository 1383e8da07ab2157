# Round 5: the RCCL path of bench.py at N = 1 (XRS_BENCH_DIST=1: process
# group over nccl = RCCL, barriers, all_reduce / all_gather of the timing)
# under torch.distributed.run, as the driver launches the multi-GPU runs.
#   bash scripts/gpu_r05_t.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05t}; mkdir -p $O
XRS_BENCH_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 1 --warmup 3 --steps 10 --no-cpu-baseline --no-f64 --no-traffic > $O/bench_rccl1.json 2> $O/bench_rccl1.err || { tail -20 $O/bench_rccl1.err; exit 1; }
cut -c1-400 $O/bench_rccl1.json
