# HBM traffic of K3i at config 3 (FETCH_SIZE / WRITE_SIZE in separate passes).
export TMPDIR=/tmp; O=gpurun_out/pmc3; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f -o f -- python3 scripts/bench_configs.py --configs 3 --cpu-seconds 0.1 --steps 1 --warmup 0 > $O/f.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w -o w -- python3 scripts/bench_configs.py --configs 3 --cpu-seconds 0.1 --steps 1 --warmup 0 > $O/w.log 2>&1
