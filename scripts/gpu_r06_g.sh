# Round 6, seventh pass: K3d (the generic coarsen, one output pixel per lane)
# and K3i / K3w gated on scale 1: the affine / coarsen suites (with the K3d
# parity test), the coarsen timings (aligned, fractional, the generic kernel
# forced onto the aligned grid, a 3.5x downscale) with kernel stats.
#   bash scripts/gpu_r06_g.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06g}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_affine_gpu.py tests/test_coarsen_gpu.py tests/test_sharding_gpu.py tests/test_multidevice_gpu.py tests/test_spatial_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { echo "pytest status $rc"; exit $rc; }
for pass in 1 2; do
  for mode in "" --frac --generic --s35; do
    timeout -k 10 120 python -u scripts/time_coarsen.py $mode 2>&1 | grep -v amdgpu.ids >> $O/coarsen.log || exit 1
    tail -1 $O/coarsen.log
  done
done
for mode in --s35 --generic; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks$mode -o ks -- python3 scripts/time_coarsen.py $mode > $O/ks$mode.log 2>&1 || exit $?
  echo "kernels $mode"; python3 scripts/kstats.py $(find $O/ks$mode -name "*kernel_stats.csv" | head -1) xrs
done
timeout -k 10 200 python -u scripts/pmc_kernels.py --counters SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_SALU --kernels affine_k3d_kernel -- scripts/time_coarsen.py --s35 > $O/pmc_k3d_s35.json 2> $O/pmc_k3d_s35.err || exit $?
cut -c1-400 $O/pmc_k3d_s35.json
