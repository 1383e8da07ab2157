# K1 probe arms: parity tests on the first arm, then the bench A/B of all.
#   bash scripts/gpu_k1arms.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
XRS_LIBRARY=probe/$1/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py tests/test_sharding_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$1.log 2>&1 || { tail -30 $O/pytest_$1.log; exit 1; }
echo "$1: $(tail -1 $O/pytest_$1.log)"
SKIP_TESTS=1 bash scripts/gpu_suite3.sh $O/ab "$@"
