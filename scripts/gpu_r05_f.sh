# Round 5: K1 work shapes whose plain copy runs >= 5.8 TB/s (profiles/
# r03_region_copy.jsonl: 1024 columns x 1 row, one float4 per thread, 6.2
# TB/s) — probe arms of the product kernel with 1024 x 1 (k1row), 512 x 1
# (k1r1p2), 1024 x 4 (k1r4n) and 1024 x 8 (k1r8n) items in plain block order
# (each XCD then holds the same column strips of every row), timed
# interleaved with the product at config 5 (checksums must agree); first the
# multi-device GPU tests.
#   bash scripts/gpu_r05_f.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05f}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_multidevice_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_md.log 2>&1; rc=$?
tail -2 $O/pytest_md.log
case $rc in 0|1) ;; *) echo "pytest status $rc"; exit $rc;; esac
for pass in 1 2; do
  for arm in base k1row k1r1p2 k1r4n k1r8n; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/k1_pad_ab.py --pad-mb 0 --tag $arm >> $O/ab.jsonl 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.jsonl
  done
done
