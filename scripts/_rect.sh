set -e
export TMPDIR=/tmp
O=gpurun_out/rect; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py tests/test_streaming_gpu.py tests/test_integration_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || true
tail -3 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c4 -- python3 scripts/bench_configs.py --configs 4 --cpu-seconds 0.2 --steps 5 > $O/c4.log 2>&1
cut -c1-300 $O/c4.log
