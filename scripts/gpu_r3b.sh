# Round-3 re-entry check: GPU suite, smoke, bench with the driver's settings,
# the RCCL (nccl backend) path of bench.py rehearsed at N = 1 under torchrun,
# and the config-4 rectify kernel stats.
#   bash scripts/gpu_r3b.sh OUTDIR
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3b}
mkdir -p $OUT
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with status $rc"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --cpu-seconds 4 > $OUT/bench_w5.json 2> $OUT/bench_w5.err || exit $?
cut -c1-400 $OUT/bench_w5.json
XRS_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 10 --warmup 5 --no-traffic --no-cpu-baseline --no-f64 > $OUT/bench_nccl1.json 2> $OUT/bench_nccl1.err || exit $?
cut -c1-300 $OUT/bench_nccl1.json
grep -o '"ranks".*' $OUT/bench_nccl1.json | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rect -o c4 -- python3 scripts/time_rectify.py --reps 10 --fused > $OUT/rect_time.log 2>&1 || exit $?
grep "ms per" $OUT/rect_time.log
cut -d, -f1-4 $OUT/rect/c4_kernel_stats.csv | cut -c1-160 | head -8
exit $rc
