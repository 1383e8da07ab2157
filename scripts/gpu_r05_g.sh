# Round 5: K1 with 1024-column items in the product's band deal (band 8 / 16 /
# 32, 4 or 8 rows in flight; the plain-copy sweep ran 1024 x 8 at 5.52 TB/s
# against 5.40 for 512 x 32), timed interleaved with the product at config 5
# (checksums must agree).
#   bash scripts/gpu_r05_g.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05g}; mkdir -p $O
for pass in 1 2; do
  for arm in base p4b8r4 p4b16r4 p4b32r4 p4b8 p4b16; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
