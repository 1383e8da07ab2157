# K1 deal vs raster placement (round 4): the product and the XCD-contiguous
# deal probe (scripts/build_probe.sh k1cont ...) timed after padding
# allocations of several sizes, interleaved, one process per run.
#   bash scripts/gpu_k1_pad.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/k1pad}; mkdir -p $O
for pass in 1 2; do
  for pad in 0 2 64 514 1030; do
    for arm in base k1cont; do
      if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
      XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb $pad --tag $arm >> $O/pad.jsonl 2> $O/pad_${arm}_${pad}.err || exit $?
      tail -1 $O/pad.jsonl
    done
  done
done
