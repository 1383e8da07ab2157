# Config-2u A/B: transform / K1p parity tests on each probe arm, then the 2u
# lines of the product and the arms, interleaved.   bash scripts/gpu_ab_2u.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for arm in "$@"; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_transform_gpu.py tests/test_crs_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_$arm.log 2>&1 || { tail -20 $O/pytest_$arm.log; exit 1; }
  echo "$arm: $(tail -1 $O/pytest_$arm.log)"
done
for pass in 1 2; do for arm in base "$@"; do
  if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -k 10 300 python -u scripts/bench_configs.py --configs 2u --cpu-seconds 0.1 > $O/ab_${arm}_$pass.jsonl 2>/dev/null || exit 1
  python3 -c "
import json
ls=[json.loads(l) for l in open('$O/ab_${arm}_$pass.jsonl')]
print('$arm', $pass, 'tables', ls[0]['transform_ms'], ls[0]['k1_ms'], ls[0]['ms_per_step'], 'fused', ls[1]['ms_per_step'])"
done; done
