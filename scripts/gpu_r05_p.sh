# Round 5: K1 with float64 output in 1024 x 12 items (product) — the
# reproject-path GPU tests, then the float64-output launch timed alternating
# with the previous commit (probe/k1head), the config-2 line (8192², float64
# out) and the bench line (its f64_out block).
#   bash scripts/gpu_r05_p.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05p}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_sharding_gpu.py tests/test_integration_gpu.py tests/test_streaming_gpu.py tests/test_spatial_gpu.py tests/test_crs_gpu.py tests/test_multidevice_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
case $rc in 0) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base k1head; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --out-dtype f64 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
timeout -k 10 600 python -u scripts/bench_configs.py --configs 2 --cpu-seconds 4 > $O/config2.jsonl 2> $O/config2.err || { tail -20 $O/config2.err; exit 1; }
cut -c1-300 $O/config2.jsonl
timeout -k 10 600 python -u bench.py --gpus 1 --warmup 5 --steps 20 > $O/bench_w5.json 2> $O/bench_w5.err || exit $?
cut -c1-300 $O/bench_w5.json
