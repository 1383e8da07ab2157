# HBM traffic of K1 at config 5 (FETCH_SIZE / WRITE_SIZE in separate passes,
# calibrated by an identity launch) -> profiles/traffic_r01.json
export TMPDIR=/tmp; O=gpurun_out/pmc5; mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o fetch -- python3 scripts/pmc_traffic.py > $O/f.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o write -- python3 scripts/pmc_traffic.py > $O/w.log 2>&1 &&
python3 scripts/pmc_traffic.py --reduce $O
