# Round 5: the fused projection gather (K1p) addressing taps and outputs by
# 32-bit element offsets from the slice bases when they fit (probe/off32):
# reproject-path GPU tests on the arm, then the 2u paths timed alternating
# with the product.
#   bash scripts/gpu_r05_ab.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05ab}; mkdir -p $O
XRS_LIBRARY=probe/off32/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_crs_gpu.py tests/test_transform_gpu.py tests/test_sharding_gpu.py tests/test_integration_gpu.py tests/test_streaming_gpu.py tests/test_spatial_gpu.py tests/test_multidevice_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_off32.log 2>&1; rc=$?
tail -2 $O/pytest_off32.log
case $rc in 0) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base off32; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_2u.py --time --tag $arm >> $O/2u.jsonl 2> $O/2u_$arm.err || exit $?
    tail -1 $O/2u.jsonl
  done
done
