export TMPDIR=/tmp; mkdir -p gpurun_out/p4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p4 -o e0 -- python scripts/bench_configs.py --configs 4 --cpu-seconds 0.2 --steps 5 > gpurun_out/p4/e0.log 2>&1
