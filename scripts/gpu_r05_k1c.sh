# Round 5, K1 column generators (coord_mode 2): reproject-path GPU tests, then
# interleaved A/B of the product (generators), the product reading the src_x
# table (--no-xgen), the previous commit (probe/k1src, src_x per item) and
# the round-4 tree (probe/k1tab, K1a tables); then the bench line.
#   bash scripts/gpu_r05_k1c.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05k1c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_sharding_gpu.py tests/test_integration_gpu.py tests/test_streaming_gpu.py tests/test_crs_gpu.py tests/test_spatial_gpu.py tests/test_multidevice_gpu.py tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_rectify_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
# a failed test is read from the log; a timeout, abort or fault ends the call here
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base basetab k1src k1tab; do
    X=""; L=xcube-resampling_amd/lib/libxrs.so
    case $arm in basetab) X=--no-xgen;; k1src|k1tab) X=--no-xgen; L=probe/$arm/pkg/lib/libxrs.so;; esac
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm $X >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
timeout -k 10 600 python -u bench.py --gpus 1 --warmup 5 --steps 20 > $O/bench_w5.json 2> $O/bench_w5.err || exit $?
cut -c1-300 $O/bench_w5.json
