# Round 6, twenty-fourth pass: the product with the per-lane claim on 8x the
# resident blocks (gpu_r06_w.sh cl8: claim 466-472 vs 505 us); 16x (cl16), and
# 16x with 8-row strips (sh8cl16: timing and checksums only, the host-tile
# path's strip count is the product's).
#   bash scripts/gpu_r06_x.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06x}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_product.log 2>&1 || { tail -5 $O/pytest_product.log; exit 1; }
echo "product parity: $(tail -1 $O/pytest_product.log)"
ARMS="cl16 sh8cl16"
for arm in cl16; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for interp in nearest bilinear; do
  for pass in 1 2 3; do
    for arm in product $ARMS; do
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
  XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 10 --res-div 2 > $O/t2_${arm}.log 2>&1 || exit $?
  echo "$arm res/2 $(grep 'ms per' $O/t2_${arm}.log)"
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm nearest"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
