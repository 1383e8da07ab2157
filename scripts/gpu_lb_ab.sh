# Rectify suite (dataset fusion for every interpolation), K4 grid arms, config-4 line.
export TMPDIR=/tmp
OUT=gpurun_out/lb
mkdir -p $OUT
true

for pass in 1 2; do
  for arm in product clb5 rlb5 rlb6; do
    if [ $arm = product ]; then L=""; else L=$PWD/probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_rectify.py --reps 20 --fused >> $OUT/ab.log 2>&1 || exit $?
  done
done
grep "ms per" $OUT/ab.log
