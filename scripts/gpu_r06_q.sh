# Round 6, seventeenth pass.  (1) K1 with 2 / 4 consecutive items of its XCD's
# sequence per block (k1p2, k1p4; no prefetch, 117 VGPRs as the product): the
# timeline (r06p) shows a median 2.1 us (mean 3.3) between an item's last
# stores and the next item's start on the same CU, ~3 of 4 block slots
# occupied; a block that runs on to its next item pays that once per P items.
# (2) K4's grid: one 64 x 16 block per wave, no cap (k4g1), or 1024 blocks
# (k4g4) instead of 2048 (a tail of waves with 3 blocks against 2).
# (3) the resolve's speculative taps with 2 rows per thread and the nearest tap
# picked by selects (spec2rb; gpu_r06_o.sh's nearest arms used scratch), its
# control p2r (the product with 2 rows).
#   bash scripts/gpu_r06_q.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06q}; mkdir -p $O
for arm in k1p2 k1p4; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_sharding_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for arm in k4g1 k4g4 spec2rb; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for out in f32 f64; do
  for pass in 1 2 3; do
    for arm in product k1p2 k1p4; do
      L=xcube-resampling_amd/lib/libxrs.so
      [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
      XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/k1_pad_ab.py --steps 30 --tag $arm --out-dtype $out >> $O/k1_items_ab.jsonl 2> $O/k1_err.log || { tail $O/k1_err.log; exit 1; }
      tail -1 $O/k1_items_ab.jsonl
    done
  done
done
for pass in 1 2 3; do
  for arm in product k4g1 k4g4 spec2rb p2r; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 > $O/t_${arm}_$pass.log 2>&1 || exit $?
    echo "$arm $pass $(grep 'ms per' $O/t_${arm}_$pass.log)"
  done
done
for arm in product k4g1 k4g4 spec2rb p2r; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm nearest"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
