set -e
export TMPDIR=/tmp
O=gpurun_out/stream2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || true
tail -3 $O/pytest.log
timeout -k 10 200 python -u scripts/bench_configs.py --configs 3 --cpu-seconds 0.5 > $O/c3.log 2>&1
cat $O/c3.log
