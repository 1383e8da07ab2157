set -e
export TMPDIR=/tmp
O=gpurun_out/k1ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_reproject_gpu.py tests/test_streaming_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || true
tail -3 $O/pytest.log
timeout -k 10 400 python -u scripts/ab_reproject.py --variants 12,23,24 --rounds 5 > $O/ab.log 2>&1
cat $O/ab.log
timeout -k 10 300 python -u scripts/ab_reproject.py --size 8192 --variants 12,23,24 --rounds 5 > $O/ab8k.log 2>&1
cat $O/ab8k.log
