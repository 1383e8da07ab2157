# Round 5: the N = 8 bench path under torch.distributed.run with gloo ranks
# sharing the one GPU (the driver's 8-GPU layout minus RCCL: the 8-way band
# split, barriers, the gathered timings; not a scaling number).
#   bash scripts/gpu_r05_aa.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05aa}; mkdir -p $O
XRS_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29688 bench.py --gpus 8 --warmup 3 --steps 5 --no-cpu-baseline --no-f64 > $O/bench_gloo8.json 2> $O/bench_gloo8.err || { tail -20 $O/bench_gloo8.err; exit 1; }
grep '^{' $O/bench_gloo8.json | cut -c1-600
