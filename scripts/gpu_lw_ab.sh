# Claim lane-window arms (probe builds) against the product at config 4.
export TMPDIR=/tmp
OUT=gpurun_out/lw
mkdir -p $OUT
for pass in 1 2; do
  for arm in product lw12 lw24; do
    if [ $arm = product ]; then L=""; else L=$PWD/probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_rectify.py --reps 20 --fused >> $OUT/ab.log 2>&1 || exit $?
  done
done
grep "ms per" $OUT/ab.log
