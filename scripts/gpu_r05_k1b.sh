# Round 5, K1 bytes vs time: the product (x entries from src_x, 8 B/column),
# the round-4 tree (probe/k1tab: K1a tables, 16 B/column) and an attribution
# probe that reads no x coordinate (probe/k1nox: src_x[c] replaced by the
# linear formula through src_x[0], src_x[1] — same taps up to rounding, values
# not bit-exact): interleaved timings, then each arm's bench line with its
# size-resolved PMC traffic.
#   bash scripts/gpu_r05_k1b.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05k1b}; mkdir -p $O
for pass in 1 2 3; do
  for arm in base k1nox k1tab; do
    if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
for arm in base k1nox k1tab; do
  if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -k 10 400 python -u bench.py --gpus 1 --warmup 5 --steps 20 --no-cpu-baseline --no-f64 > $O/bench_$arm.json 2> $O/bench_$arm.err || exit $?
  cut -c1-200 $O/bench_$arm.json
done
