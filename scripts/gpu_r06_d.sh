# Round 6, fourth pass: K3w arms (one output row per item; 4 waves per SIMD by
# launch bounds) for parity and interleaved timing on the fractional coarsen;
# resolve arms with 2-D items (128 columns x 12 rows; 5 / 6 waves per SIMD)
# for parity, timing, kernel stats and read traffic; then every config line.
#   bash scripts/gpu_r06_d.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06d}; mkdir -p $O
for arm in k3wr1 k3wlb4; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_affine_gpu.py -m gpu -q -x -k "k3w or integral" --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for pass in 1 2 3; do
  for arm in product k3wr1 k3wlb4; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_coarsen.py --frac 2>&1 | grep -v amdgpu.ids >> $O/coarsen.log || exit 1
    tail -1 $O/coarsen.log
  done
done
ARMS="r2d r2d6"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
for pass in 1 2 3; do
  for arm in product $ARMS; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 > $O/t_${arm}_$pass.log 2>&1 || exit $?
    echo "$arm $pass $(grep 'ms per' $O/t_${arm}_$pass.log)"
  done
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 20 > $O/ks_$arm.log 2>&1 || exit $?
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) resolve
  XRS_LIBRARY=$L timeout -k 10 200 python -u scripts/pmc_kernels.py --counters TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum --kernels resolve -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_rd_$arm.json 2> $O/pmc_rd_$arm.err || exit $?
  cut -c1-200 $O/pmc_rd_$arm.json
done
# the generic K3 (forced on the aligned grid; and a 3.5x downscale, div-x
# grid at scale 0.875): time and one PMC pass each
for mode in --generic --s35; do
  timeout -k 10 120 python -u scripts/time_coarsen.py $mode 2>&1 | grep -v amdgpu.ids >> $O/coarsen.log || exit 1
  tail -1 $O/coarsen.log
  timeout -k 10 200 python -u scripts/pmc_kernels.py --counters SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES --kernels affine_reduce_kernel,integral_finish,affine_reduce_integral -- scripts/time_coarsen.py $mode > $O/pmc_k3$mode.json 2> $O/pmc_k3$mode.err || exit $?
  cut -c1-600 $O/pmc_k3$mode.json
done
timeout -k 10 1000 python -u scripts/bench_configs.py --configs 1,2,2u,3,3f,4 --cpu-seconds 6 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cut -c1-200 $O/configs.jsonl
