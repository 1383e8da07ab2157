# Round-3 new/changed GPU tests, then the K1 shape A/B and a --warmup 5 bench.
export TMPDIR=/tmp
O=${1:-gpurun_out/r3a}; shift; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_sharding_gpu.py "tests/test_configs_gpu.py::test_config2_reproject_bilinear_8192_f64" "tests/test_affine_gpu.py::test_config3_full_size_sampled_blocks" "tests/test_transform_gpu.py::test_streamed_host_source_fuses_when_tables_exceed_budget" -x -v --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1 || { tail -40 $O/pytest_new.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/pytest_new.log | tail -12
