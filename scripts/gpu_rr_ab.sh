# Resolve rows-per-item arms (probe builds) against the product at config 4.
export TMPDIR=/tmp
OUT=gpurun_out/rr
mkdir -p $OUT
for pass in 1 2; do
  for arm in product rr2 rr3 rr6 sh8 sh32; do
    if [ $arm = product ]; then L=""; else L=$PWD/probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_rectify.py --reps 20 --fused >> $OUT/ab.log 2>&1 || exit $?
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_rectify.py --reps 20 >> $OUT/ab.log 2>&1 || exit $?
  done
done
grep "ms per" $OUT/ab.log
