export TMPDIR=/tmp
OUT=gpurun_out/k1a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic --no-f64 > $OUT/bench.json 2> $OUT/bench.err || exit $?
cut -c1-400 $OUT/bench.json
timeout -k 10 300 python -u scripts/rehearse_bands.py > $OUT/bands.jsonl 2> $OUT/bands.err || exit $?
python -c "
import json
for l in open('$OUT/bands.jsonl'):
    d=json.loads(l); print(d['world'], d['balance'], d['max_ms'], d['max_over_mean'], [r['ms'] for r in d['ranks']])
"
