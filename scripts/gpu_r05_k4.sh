# Round 5, K4 (ij_bboxes_block_kernel) arms at config 4: 4 waves per SIMD by
# launch bounds (k4lb4), one 64x16 block per wave (k4grid: grid cap 256 x 64
# blocks), both (k4both) — timed interleaved (K4 + K5 + K6 fused nearest),
# then each arm's kernel stats.
#   bash scripts/gpu_r05_k4.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05k4}; mkdir -p $O
ARMS="base k4lb4 k4grid k4both"
for pass in 1 2 3; do
  for arm in $ARMS; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 >> $O/ab.log 2> $O/ab_$arm.err || exit $?
    tail -1 $O/ab.log
  done
done
for arm in $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
