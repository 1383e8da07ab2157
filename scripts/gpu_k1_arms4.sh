# K1b column-group deal (round 4): reproject parity on the product library,
# then bench A/B interleaved (product = column groups of 4 segments; probe
# arms: k1ntld = nt-hinted tap loads, k1cg16/20 = column groups), then
# the size-resolved read traffic of the product and of k1old.
#   bash scripts/gpu_k1_colgroup.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/k1cg}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_sharding_gpu.py tests/test_streaming_gpu.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="bench.py --no-cpu-baseline --no-traffic --steps 30 --warmup 10"
for pass in 1 2; do
  for arm in base k1ntld k1cg16 k1cg20; do
    if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 300 python -u $B > $O/ab_${arm}_$pass.json 2> $O/ab_${arm}_$pass.err || exit $?
    python -c "import json; d=json.load(open('$O/ab_${arm}_$pass.json')); print('$arm', $pass, d['roofline']['kernel_ms'], d['ms_per_step'], d['f64_out']['kernel_ms'])"
  done
done
for arm in base k1ntld; do
  if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d $O/pmc_$arm/rd -o rd -- python3 scripts/pmc_traffic.py > $O/pmc_$arm.log 2>&1 || exit $?
  XRS_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d $O/pmc_$arm/wr -o wr -- python3 scripts/pmc_traffic.py >> $O/pmc_$arm.log 2>&1 || exit $?
  python scripts/pmc_traffic.py --reduce $O/pmc_$arm > $O/traffic_$arm.json || exit $?
  python -c "import json; d=json.load(open('$O/traffic_$arm.json')); print('$arm', {k: (v['read_bytes'], v.get('read_over_known')) for k, v in d['launches'].items()})"
done
