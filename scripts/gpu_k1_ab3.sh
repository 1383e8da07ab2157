# K1 round-3 A/B: reproject GPU tests on the product library, then the bench
# (f32 and f64 out) for the product and probe arms, interleaved.
#   bash scripts/gpu_k1_ab3.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_transform_gpu.py tests/test_streaming_gpu.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="bench.py --no-cpu-baseline --no-traffic --steps 30 --warmup 30"
for pass in 1 2; do
  for arm in base "$@"; do
    if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 300 python -u $B > $O/ab_${arm}_$pass.json 2> $O/ab_${arm}_$pass.err || exit $?
    python -c "import json; d=json.load(open('$O/ab_${arm}_$pass.json')); print('$arm', $pass, d['roofline']['kernel_ms'], d['ms_per_step'], d['f64_out']['kernel_ms'])"
  done
done
