# Round 5, K2 grouped items: affine / multidevice GPU tests, then the config-1
# single and batched (64 x 1024^2) launches timed interleaved against the
# previous kernel (probe/k2old), then the K1 bench line once more.
#   bash scripts/gpu_r05_k2.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05k2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_multidevice_gpu.py tests/test_configs_gpu.py tests/test_integration_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2 3; do
  for arm in base k2old; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_affine.py --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
