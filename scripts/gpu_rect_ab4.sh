# Rectify (config 4) round 4: rectify parity tests on the product library,
# then K4 + K5 + K6 timing interleaved for the product and probe arms, and the
# product's kernel stats.   bash scripts/gpu_rect_ab4.sh OUTDIR ARM...
export TMPDIR=/tmp
O=${1:-gpurun_out/rab}; shift; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py tests/test_gridmapping_goldens_gpu.py tests/test_sharding_gpu.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for pass in 1 2 3; do
  for arm in product "$@"; do
    P=""
    if [ $arm = product ]; then L=""; elif [ -d probe/$arm/root ]; then L=""; P=$PWD/probe/$arm/root; else L=$PWD/probe/$arm/pkg/lib/libxrs.so; fi
    XRS_PYROOT=$P XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_rectify.py --reps 20 --fused > $O/t_${arm}_$pass.log 2>&1 || exit $?
    echo "$arm $pass $(grep 'ms per' $O/t_${arm}_$pass.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c4 -- python3 scripts/time_rectify.py --reps 10 --fused > $O/prof.log 2>&1 || exit $?
python scripts/kstats.py $O/prof/c4_kernel_stats.csv | head -8
