# Config-line A/B: the product library against probe builds (probe/<name>),
# interleaved twice.   bash scripts/gpu_ab_configs.sh OUTDIR CONFIGS ARM [ARM ...]
export TMPDIR=/tmp
OUT=$1; C=$2; shift 2
mkdir -p $OUT
for pass in 1 2; do
  for arm in base "$@"; do
    if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 300 python -u scripts/bench_configs.py --configs $C --cpu-seconds 0.1 > $OUT/ab_${arm}_$pass.jsonl 2> $OUT/ab_${arm}_$pass.err || exit $?
    python -c "
import json
for l in open('$OUT/ab_${arm}_$pass.jsonl'):
    d=json.loads(l); print('$arm', $pass, d['config'], d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
