# Round 4: the new parity tests (fused rectify at config 4, config 2 all tiles,
# host register / staging threads) and the bench launcher on a 1-GPU box.
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_streaming_gpu.py::test_host_register_copy_unregister_then_fresh_pageable_copy" \
  "tests/test_streaming_gpu.py::test_staging_concurrent_threads" \
  "tests/test_streaming_gpu.py::test_staging_round_trip_multi_chunk" \
  "tests/test_rectify_gpu.py::test_config4_full_size_matches_oracle" \
  "tests/test_rectify_gpu.py::test_rectify_dataset_fused_first_variable" \
  tests/test_configs_gpu.py > $OUT/pytest_items.log 2>&1 || { tail -30 $OUT/pytest_items.log; exit 1; }
tail -3 $OUT/pytest_items.log
rc=0
timeout -k 10 120 python -u bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/bench_g2.json 2> $OUT/bench_g2.err || rc=$?
echo "bench --gpus 2 on one GPU: rc=$rc"; tail -2 $OUT/bench_g2.err
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_g1.json 2> $OUT/bench_g1.err || exit $?
cut -c1-300 $OUT/bench_g1.json
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps(d['roofline']))" $OUT/bench_g1.json
timeout -k 10 200 python -u scripts/xcd_probe.py > $OUT/xcd_probe.jsonl 2> $OUT/xcd_probe.err || exit $?
python - $OUT/xcd_probe.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[r["chunk"]].append(r["GBs"])
for k, v in d.items():
    print(k, min(v), max(v))
PY
