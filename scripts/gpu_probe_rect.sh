# Rectify probe arms: the rectify GPU tests on each probe library, then the
# config-4 kernel timing A/B (scripts/gpu_rect3.sh).   bash scripts/gpu_probe_rect.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for arm in "$@"; do
  [ "$arm" = fused ] && continue
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$arm.log 2>&1 || { tail -30 $O/pytest_$arm.log; exit 1; }
  echo "$arm: $(tail -1 $O/pytest_$arm.log)"
done
bash scripts/gpu_rect3.sh $O/rect "$@"
