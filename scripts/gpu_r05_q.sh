# Round 5: float32-output K1 shapes around the product (512 x 32, 8 rows in
# flight): 4 rows in flight (6 waves per SIMD), 16 rows (2 waves), 24-row
# bands, and the float64 winner 1024 x 12 (4 rows), each alternating with
# the product at config 5 (checksums must agree).
#   bash scripts/gpu_r05_q.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05q}; mkdir -p $O
for pass in 1 2 3; do
  for arm in base f2b32r4 base f4b12r4 base f2b24r8 base f2b32r16; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
