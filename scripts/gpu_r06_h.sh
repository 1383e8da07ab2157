# Round 6, eighth pass: the generic K3's phase A with the tile's sub-samples
# batched in row-major order across its output rows (product: 2 at a time;
# arms flat4 / flat8): the affine / coarsen suites on each, then interleaved
# timings of the generic kernel (forced onto the aligned grid; a 3.5x
# downscale) and of the aligned / fractional fast paths.
#   bash scripts/gpu_r06_h.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06h}; mkdir -p $O
for arm in product flat4 flat8; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for pass in 1 2; do
  for arm in product flat4 flat8; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    for mode in --generic --s35; do
      XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_coarsen.py $mode 2>&1 | grep -v amdgpu.ids >> $O/coarsen.log || exit 1
      tail -1 $O/coarsen.log
    done
  done
done
for mode in "" --frac; do
  timeout -k 10 120 python -u scripts/time_coarsen.py $mode 2>&1 | grep -v amdgpu.ids >> $O/coarsen.log || exit 1
  tail -1 $O/coarsen.log
done
