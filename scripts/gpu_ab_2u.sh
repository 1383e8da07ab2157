export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_transform_gpu.py tests/test_crs_gpu.py tests/test_reproject_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/k1c.log 2>&1; tail -1 gpurun_out/k1c.log
for pass in 1 2; do for arm in base k1c_orig k1c_r2; do
  if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -k 10 300 python -u scripts/bench_configs.py --configs 2u --cpu-seconds 0.1 > gpurun_out/ab12_${arm}_$pass.jsonl 2>/dev/null || exit $?
  python3 -c "
import json
d=json.loads(open('gpurun_out/ab12_${arm}_$pass.jsonl').readline()); print('$arm', $pass, d['k1_ms'], d['transform_ms'], d['ms_per_step'])"
done; done
