# Claim / resolve / K4 kernel times of probe arms (attribution builds,
# scripts/build_probe.sh) next to the product, one rocprofv3 --stats run each.
#   bash scripts/gpu_rect_kstats_arms.sh OUTDIR ARM...
export TMPDIR=/tmp
O=${1:-gpurun_out/karms}; shift; mkdir -p $O
for arm in product "$@"; do
  if [ $arm = product ]; then L=""; else L=$PWD/probe/$arm/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$arm -o k -- python3 scripts/time_rectify.py --reps 10 --fused > $O/$arm.log 2>&1 || exit $?
  echo "$arm $(grep 'ms per' $O/$arm.log | sed 's/.*: //')"
  python3 scripts/kstats.py $O/$arm/k_kernel_stats.csv > $O/$arm.kstats 2>&1
  grep -E "claim|resolve|bboxes" $O/$arm.kstats
done
