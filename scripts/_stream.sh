set -e
export TMPDIR=/tmp
O=gpurun_out/stream; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_streaming_gpu.py tests/test_reproject_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || true
tail -3 $O/pytest.log
timeout -k 10 400 python -u scripts/bench_host.py > $O/host.jsonl 2> $O/host.err
cat $O/host.jsonl
