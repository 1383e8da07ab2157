# Round 5: K1 1024-column items around the 16-row band (the first sweep,
# gpu_r05_g.sh: 1024 x 16 with 4 rows in flight 2.508 vs 2.52 ms for the
# product 512 x 32), and 2048-column items, timed interleaved at config 5
# (checksums must agree).
#   bash scripts/gpu_r05_h.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05h}; mkdir -p $O
for pass in 1 2 3; do
  for arm in base p4b16r4 p4b12r4 p4b20r4 p4b24r4 p8b8r2 p8b16r2; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
