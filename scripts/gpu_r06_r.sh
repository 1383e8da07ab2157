# Round 6, eighteenth pass: K4's grid at the resident block count (k4res:
# resident_blocks(), 1024 on MI355X; gpu_r06_q.sh's k4g4 = 1024 blocks ran K4
# 96.2 vs 101.4 us), with 8-row wave blocks (k4res8), at 768 blocks (k4g3),
# and k4res with the resolve at 2 rows per thread (k4resp2); the claim's
# strips at 8 / 12 / 24 quad rows instead of 16 (sh8, sh12, sh24: timing and
# checksums only — the host-tile path's strip count is the product's).
#   bash scripts/gpu_r06_r.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06r}; mkdir -p $O
ARMS="k4res k4res8 k4g3 k4resp2"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for interp in nearest bilinear; do
  for pass in 1 2 3; do
    for arm in product $ARMS sh8 sh12 sh24; do
      L=xcube-resampling_amd/lib/libxrs.so
      [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
      XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 --interp $interp > $O/t_${arm}_${interp}_$pass.log 2>&1 || exit $?
      echo "$arm $interp $pass $(grep 'ms per' $O/t_${arm}_${interp}_$pass.log)"
    done
  done
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm nearest"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
