# Round 6, sixteenth pass: (1) K1's item timeline (probe/k1tl, scripts/k1_timeline.py:
# per CU, the time an item's prologue is exposed, i.e. no item of the CU
# streams taps) for VERDICT r05 item 2; (2) the claim's per-lane row
# reciprocal by v_rcp_f32 instead of an IEEE division (crcp); (3) the resolve
# with 2 rows per thread (p2r, the control of gpu_r06_o.sh) again, with stats.
#   bash scripts/gpu_r06_p.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06p}; mkdir -p $O
for pass in 1 2; do
  XRS_LIBRARY=probe/k1tl/pkg/lib/libxrs.so timeout -k 10 240 python -u scripts/k1_timeline.py $O/k1_timeline_$pass.json > $O/k1tl_$pass.log 2>&1 || { tail -20 $O/k1tl_$pass.log; exit 1; }
  tail -1 $O/k1tl_$pass.log
done
ARMS="crcp p2r"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for pass in 1 2 3; do
  for arm in product $ARMS; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 > $O/t_${arm}_$pass.log 2>&1 || exit $?
    echo "$arm $pass $(grep 'ms per' $O/t_${arm}_$pass.log)"
  done
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm nearest"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
