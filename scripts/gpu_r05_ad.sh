# Round 5: config 3's two small kernels — run records by a wave ballot in the
# tables kernel (product now; probe/k3head = previous commit), and the finish
# kernel on a grid capped at 1024 / 512 blocks (probe/fin1024, fin512; the
# generic fallback it carries is grid-stride): affine / coarsen GPU tests on
# the product and fin1024, config 3 timed alternating, kernel stats.
#   bash scripts/gpu_r05_ad.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05ad}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_configs_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_base.log 2>&1; rc=$?
tail -1 $O/pytest_base.log
case $rc in 0) ;; *) echo "pytest status $rc"; exit $rc;; esac
XRS_LIBRARY=probe/fin1024/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_configs_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_fin1024.log 2>&1; rc=$?
tail -1 $O/pytest_fin1024.log
case $rc in 0) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in k3head base fin1024 base fin512; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_coarsen.py >> $O/k3_ab.log 2> $O/k3_ab_$arm.err || exit $?
    echo "$arm $(tail -1 $O/k3_ab.log)"
  done
done
for arm in base fin1024; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_coarsen.py > $O/ks_$arm.log 2>&1 || exit $?
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) integral finish tables
done
