# Round 5: K1 with raised wave priority while a batch's tap loads issue
# (s_setprio 1 or 3 around the loads, back to 0 — or 1 — before the
# deferred stores), alternating with the product at config 5.
#   bash scripts/gpu_r05_r.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05r}; mkdir -p $O
for pass in 1 2 3; do
  for arm in base prio1 base prio3 base prio3s; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
