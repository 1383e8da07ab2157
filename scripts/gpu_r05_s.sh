# Round 5: K1 cache policies — plain instead of non-temporal stores
# (plainst), tap loads with the slc / nt bit (ldslc) or glc / sc0 (ldglc) —
# alternating with the product at config 5 (checksums must agree).
#   bash scripts/gpu_r05_s.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05s}; mkdir -p $O
for pass in 1 2 3; do
  for arm in base plainst base ldslc base ldglc; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
