# K1 LDS-image arm: parity tests on the probe library, product transform /
# rectify tests, rectify fused A/B, config 2u, then K1 bench A/B (product vs
# probe arms).   bash scripts/gpu_r3c.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for arm in "$@"; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_sharding_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$arm.log 2>&1 || { tail -30 $O/pytest_$arm.log; exit 1; }
  echo "$arm: $(tail -1 $O/pytest_$arm.log)"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
echo "product suite: $(tail -1 $O/pytest_gpu.log)"
bash scripts/gpu_rect3.sh $O/rect fused || exit 1
timeout -k 10 300 python -u scripts/bench_configs.py --configs 2u --cpu-seconds 1 > $O/c2u.jsonl 2> $O/c2u.err || exit 1
python -c "import json; [print(d['config'], d['ms_per_step'], d['roofline']['kernel']) for d in map(json.loads, open('$O/c2u.jsonl'))]"
SKIP_TESTS=1 bash scripts/gpu_suite3.sh $O/ab "$@"
