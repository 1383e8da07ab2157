# K1 A/B: the product library against timing-probe builds (probe/<name>, made
# by scripts/build_probe.sh), interleaved so box drift shows; then the rectify
# kernel stats and the two PMC passes of scripts/pmc_rectify.sh.
#   bash scripts/gpu_ab_k1.sh OUTDIR ARM [ARM ...]
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="bench.py --no-cpu-baseline --no-traffic --no-f64 --steps 30"
for pass in 1 2; do
  for arm in base "$@"; do
    if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 300 python -u $B > $OUT/ab_${arm}_$pass.json 2> $OUT/ab_${arm}_$pass.err || exit $?
    python -c "import json,sys; d=json.load(open('$OUT/ab_${arm}_$pass.json')); print('$arm', $pass, d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
