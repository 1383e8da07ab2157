# Round 6, third pass: K3w (fractional-offset coarsen: contiguous runs with
# weights) parity in the affine / coarsen suites and its timing against round
# 5 (generic K3) on a 16384^2 -> 4096^2 4x4 mean whose target is shifted by
# 0.3 source pixels, plus the aligned config 3; resolve arms that deal groups
# of 8 / 32 consecutive bands to each XCD (parity, interleaved timing, kernel
# stats, L2 -> fabric read requests per kernel).
#   bash scripts/gpu_r06_c.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_native_abi.py tests/test_multidevice_gpu.py tests/test_sharding_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_affine.log 2>&1; rc=$?
tail -3 $O/pytest_affine.log
[ $rc -eq 0 ] || { echo "pytest status $rc"; exit $rc; }
for pass in 1 2; do
  for arm in product r5; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_coarsen.py --frac 2>&1 | grep -v amdgpu.ids >> $O/coarsen.log || exit 1
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_coarsen.py 2>&1 | grep -v amdgpu.ids >> $O/coarsen.log || exit 1
    tail -2 $O/coarsen.log
  done
done
ARMS="rxg8 rxg32"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x -k "config4_full or fused_resolve or triangle_keys" --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
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
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 20 > $O/ks_$arm.log 2>&1 || exit $?
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
  XRS_LIBRARY=$L timeout -k 10 200 python -u scripts/pmc_kernels.py --counters TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum --kernels resolve -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_rd_$arm.json 2> $O/pmc_rd_$arm.err || exit $?
  cut -c1-300 $O/pmc_rd_$arm.json
done
