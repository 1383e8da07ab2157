# Round 5: the float64-output K1 line (the reference's bilinear dtype) —
# work shapes with the round-5 prologue: (columns per thread, band rows,
# rows in flight) = product (4, 8, 4) against (4, 16, 4), (4, 4, 4),
# (4, 12, 4), (2, 8, 4), (2, 16, 4), (2, 32, 4), (2, 32, 8), timed
# interleaved at config 5 with float64 output (checksums must agree); the
# second form alternates the product with each arm.
#   bash scripts/gpu_r05_o.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05o}; mkdir -p $O
for pass in 1 2 3; do
  for arm in base q4b12r4 base q2b16r4 base q4b16r4 base q2b32r8; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --out-dtype f64 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
