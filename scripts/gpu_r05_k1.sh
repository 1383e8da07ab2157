# Round 5, K1 with in-item axis entries: the GPU suite, an interleaved A/B
# against the round-4 tree (probe/k1tab, scripts/build_rev.sh k1tab <rev>),
# and the bench line with its PMC traffic passes.
#   bash scripts/gpu_r05_k1.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05k1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for pass in 1 2 3; do
  for arm in base k1tab; do
    if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
timeout -k 10 600 python -u bench.py --gpus 1 --warmup 5 --steps 20 > $O/bench_w5.json 2> $O/bench_w5.err || exit $?
cut -c1-400 $O/bench_w5.json
