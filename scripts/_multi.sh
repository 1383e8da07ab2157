set -e
export TMPDIR=/tmp
O=gpurun_out/multi; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_spatial_gpu.py tests/test_integration_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || true
tail -3 $O/pytest.log
timeout -k 10 200 python -u scripts/bench_configs.py --configs 1 --cpu-seconds 1 > $O/c1.log 2>&1
cat $O/c1.log
XRS_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > $O/b2.json 2> $O/b2.err
cat $O/b2.json
XRS_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --shard bands > $O/b2b.json 2> $O/b2b.err
cat $O/b2b.json
