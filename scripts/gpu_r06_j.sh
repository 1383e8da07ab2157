# Round 6, tenth pass: claim windows above kLaneWindow walked by the wave on
# the quad's forms (product) against the exact big-window walk it replaces
# (head) and the wave-compacted claim walk on that tree (compact), at
# config 4 and at finer targets (--res-div 1.5 / 2 / 3: larger windows); the
# rectify suite on each first, then claim kernel stats.
#   bash scripts/gpu_r06_j.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06j}; mkdir -p $O
ARMS="head compact"
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for div in 1 1.5 2 3; do
  for pass in 1 2; do
    for arm in product $ARMS; do
      L=xcube-resampling_amd/lib/libxrs.so
      [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
      XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 10 --res-div $div > $O/t_${arm}_${div}_$pass.log 2>&1 || exit $?
      echo "$arm $pass $(grep 'ms per' $O/t_${arm}_${div}_$pass.log)"
    done
  done
done
for div in 1 2; do
  for arm in product $ARMS; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_${arm}_$div -o ks -- python3 scripts/time_rectify.py --fused --reps 10 --res-div $div > $O/ks_${arm}_$div.log 2>&1 || exit $?
    echo "$arm res/$div"; python3 scripts/kstats.py $(find $O/ks_${arm}_$div -name "*kernel_stats.csv" | head -1) rectify
  done
done
