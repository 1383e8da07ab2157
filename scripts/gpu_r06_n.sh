# Round 6, fourteenth pass: the compacted claim walk with fewer fetches per
# step — c2: the window origin as one packed word and the owner's reciprocal
# recomputed (2 ds_bpermute per step instead of 4); c3: c2 with each lane's
# forms as 64 contiguous LDS bytes read by 4 b128 loads (instead of 8 b64).
# The rectify suite on each, then interleaved timing (compacted walk forced
# at config 4, the product's choice at 2x / 3x finer grids) and claim stats.
#   bash scripts/gpu_r06_n.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06n}; mkdir -p $O
ARMS="c2 c3"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for spec in "1 1" "2 0" "3 0"; do
  set -- $spec
  for pass in 1 2; do
    for arm in product $ARMS; do
      L=xcube-resampling_amd/lib/libxrs.so
      [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
      XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 10 --res-div $1 --compact $2 > $O/t_${arm}_$1_$pass.log 2>&1 || exit $?
      echo "$arm $pass $(grep 'ms per' $O/t_${arm}_$1_$pass.log)"
    done
  done
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 --res-div 2 > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm res/2"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim
done
