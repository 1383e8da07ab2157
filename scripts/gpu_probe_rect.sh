# Rectify parity tests on the product library, then config-4 kernel stats for
# the product and each probe named on the command line.
#   bash scripts/gpu_probe_rect.sh OUT [probe ...]
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py tests/test_spatial_gpu.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for p in product "$@"; do
  if [ $p = product ]; then L=xcube_resampling_amd/lib/libxrs.so; else L=probe/$p/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$p -o s -- python3 scripts/time_rectify.py --reps 10 > $O/$p.log 2>&1 || exit $?
  echo "$p $(grep -h 'ms per' $O/$p.log) | claim $(grep -h claim $O/$p/s_kernel_stats.csv | cut -d, -f4) resolve $(grep -h resolve $O/$p/s_kernel_stats.csv | cut -d, -f4)"
done
