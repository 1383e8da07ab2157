# GPU suite, then the config-line kernel stats.   bash scripts/gpu_suite_configs.sh OUTDIR [CONFIGS]
export TMPDIR=/tmp
OUT=$1; C=${2:-1,2,3,4}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash scripts/gpu_prof_configs.sh $OUT $C
