# Config 3 K3i arms (round 4): the affine / coarsen parity tests on the
# product, then every arm timed interleaved (scripts/time_coarsen.py).
#   bash scripts/gpu_k3_ab.sh OUTDIR ARM...
export TMPDIR=/tmp
O=${1:-gpurun_out/k3ab}; shift; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for pass in 1 2 3; do
  for arm in product "$@"; do
    if [ $arm = product ]; then L=""; else L=$PWD/probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_coarsen.py > $O/t_${arm}_$pass.log 2>&1 || { tail -5 $O/t_${arm}_$pass.log; exit 1; }
    echo "$arm $pass $(grep 'ms per' $O/t_${arm}_$pass.log)"
  done
done
