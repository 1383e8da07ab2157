# Round 5: config 2u with tmerc's asinh argument sqrt(tan^2 + 1) taken from
# the normalisation already computed (1 / |(sin_Cn, cos_Cn cos_Ce)|; probe/
# asinh1): transform / CRS / reproject GPU tests on the arm, then both 2u
# paths timed alternating with the product.
#   bash scripts/gpu_r05_u.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05y}; mkdir -p $O
XRS_LIBRARY=probe/asinh1/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_transform_gpu.py tests/test_crs_gpu.py tests/test_reproject_gpu.py tests/test_configs_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_asinh1.log 2>&1; rc=$?
tail -2 $O/pytest_asinh1.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base asinh1; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_2u.py --time --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
