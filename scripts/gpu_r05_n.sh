# Round 5: after the vectorised plan bounds — the reproject-path GPU tests
# and smoke on the final tree.
#   bash scripts/gpu_r05_n.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05n}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_sharding_gpu.py tests/test_integration_gpu.py tests/test_streaming_gpu.py tests/test_spatial_gpu.py tests/test_crs_gpu.py tests/test_transform_gpu.py tests/test_multidevice_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
case $rc in 0) ;; *) echo "pytest status $rc"; exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
