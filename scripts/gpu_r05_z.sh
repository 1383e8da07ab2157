# Round 5: the gathers' index division (coord - origin) / res without a
# division instruction (div_by: two FMA corrections of a * RN(1/res),
# correctly rounded; probe/divby): reproject-path GPU tests on the arm, then
# K1 (float32 and float64 output) and the fused 2u gather timed alternating
# with the product.
#   bash scripts/gpu_r05_z.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05z}; mkdir -p $O
XRS_LIBRARY=probe/divby/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_crs_gpu.py tests/test_transform_gpu.py tests/test_sharding_gpu.py tests/test_integration_gpu.py tests/test_streaming_gpu.py tests/test_spatial_gpu.py tests/test_multidevice_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_divby.log 2>&1; rc=$?
tail -2 $O/pytest_divby.log
case $rc in 0) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base divby; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/k1_f32.jsonl 2> $O/k1_f32_$arm.err || exit $?
    tail -1 $O/k1_f32.jsonl
  done
done
for pass in 1 2; do
  for arm in base divby; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --out-dtype f64 --tag $arm >> $O/k1_f64.jsonl 2> $O/k1_f64_$arm.err || exit $?
    tail -1 $O/k1_f64.jsonl
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_2u.py --time --tag $arm >> $O/2u.jsonl 2> $O/2u_$arm.err || exit $?
    tail -1 $O/2u.jsonl
  done
done
