# Round 5: after the 2u changes (32-bit index arithmetic in the per-pixel
# gathers, reciprocal products in the LAEA -> tmerc pipeline) — the whole
# GPU suite, then the 2u config lines.
#   bash scripts/gpu_r05_v.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05v}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
case $rc in 0) ;; *) echo "pytest status $rc"; exit $rc;; esac
timeout -k 10 600 python -u scripts/bench_configs.py --configs 2u --cpu-seconds 4 > $O/config2u.jsonl 2> $O/config2u.err || { tail -20 $O/config2u.err; exit 1; }
cut -c1-250 $O/config2u.jsonl
