set -e
export TMPDIR=/tmp
O=gpurun_out/k3i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_spatial_gpu.py tests/test_streaming_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || true
tail -3 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_configs.py --configs 3 --cpu-seconds 0.5 > $O/c3_k3i.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python3 scripts/bench_configs.py --configs 3 --cpu-seconds 0.2 > $O/c3_prof.log 2>&1
