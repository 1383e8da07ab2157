# Round 6, sixth pass: K3i's slow-list appends aggregated per wave (one
# atomic per wave and row): the affine / coarsen suites, then the coarsen
# timings (aligned, fractional, the generic kernel forced, a 3.5x downscale)
# with the 3.5x downscale's kernel stats, and the 2u fused reprojection
# against round 5 (the ADVICE fix's near-threshold branch).
#   bash scripts/gpu_r06_f.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06f}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_sharding_gpu.py tests/test_multidevice_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { echo "pytest status $rc"; exit $rc; }
for pass in 1 2; do
  for mode in "" --frac --generic --s35; do
    timeout -k 10 120 python -u scripts/time_coarsen.py $mode 2>&1 | grep -v amdgpu.ids >> $O/coarsen.log || exit 1
    tail -1 $O/coarsen.log
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_c -o ks -- python3 scripts/time_coarsen.py --s35 > $O/ks_c.log 2>&1 || exit $?
python3 scripts/kstats.py $(find $O/ks_c -name "*kernel_stats.csv" | head -1) xrs
for pass in 1 2 3; do
  for arm in product r5; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_2u.py --time --reps 20 --tag $arm > $O/t2u_${arm}_$pass.log 2>&1 || exit $?
    echo "$arm $pass $(tail -1 $O/t2u_${arm}_$pass.log)"
  done
done
