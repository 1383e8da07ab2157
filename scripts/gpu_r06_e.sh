# Round 6, fifth pass: the product with K3g (generic coarsen on lane groups),
# K3w at 4 waves per SIMD and the 2-D resolve items: the affine / coarsen /
# rectify / sharding / multidevice suites, then the coarsen timings (aligned
# config 3 = K3i, fractional shift = K3w, the generic kernel forced on the
# aligned grid, a 3.5x downscale = K3i overflow -> K3g) and the rectify
# timing with kernel stats.
#   bash scripts/gpu_r06_e.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06e}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_rectify_gpu.py tests/test_sharding_gpu.py tests/test_multidevice_gpu.py tests/test_spatial_gpu.py tests/test_streaming_gpu.py -m gpu -q -x --durations 5 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -8 $O/pytest.log
[ $rc -eq 0 ] || { echo "pytest status $rc"; exit $rc; }
for pass in 1 2; do
  for mode in "" --frac --generic --s35; do
    timeout -k 10 120 python -u scripts/time_coarsen.py $mode 2>&1 | grep -v amdgpu.ids >> $O/coarsen.log || exit 1
    tail -1 $O/coarsen.log
  done
done
timeout -k 10 200 python -u scripts/pmc_kernels.py --counters SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_SALU --kernels affine_lanes_kernel,integral_finish -- scripts/time_coarsen.py --s35 > $O/pmc_k3g_s35.json 2> $O/pmc_k3g_s35.err || exit $?
cut -c1-500 $O/pmc_k3g_s35.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_c -o ks -- python3 scripts/time_coarsen.py --s35 > $O/ks_c.log 2>&1 || exit $?
python3 scripts/kstats.py $(find $O/ks_c -name "*kernel_stats.csv" | head -1)
for pass in 1 2; do
  timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 > $O/t_rect_$pass.log 2>&1 || exit $?
  grep 'ms per' $O/t_rect_$pass.log
done
