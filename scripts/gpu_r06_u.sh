# Round 6, twenty-first pass: the 7-wave resolve with 16384 / 32768 / 65536
# blocks (r7g16k: 258.7 us in gpu_r06_t.sh; more blocks than items leave the
# extra ones empty), and K1 under launch bounds for 5 waves per SIMD (k1lb5:
# 96 VGPRs, 27 spilled; the timeline showed 3 of 4 item slots busy).
#   bash scripts/gpu_r06_u.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06u}; mkdir -p $O
ARMS="r7g16k r7g32k r7g64k"
for arm in r7g32k r7g64k; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
  echo "$arm parity: $(tail -1 $O/pytest_$arm.log)"
  [ $rc -eq 0 ] || { echo "$arm pytest status $rc"; exit $rc; }
done
XRS_LIBRARY=probe/k1lb5/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_reproject_gpu.py tests/test_configs_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -k "not rectify and not config4" > $O/pytest_k1lb5.log 2>&1 || { tail -5 $O/pytest_k1lb5.log; exit 1; }
echo "k1lb5 parity: $(tail -1 $O/pytest_k1lb5.log)"
for pass in 1 2; do
  for arm in product k1lb5; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/k1_pad_ab.py --steps 30 --tag $arm >> $O/k1_lb5_ab.jsonl 2> $O/k1_err.log || { tail $O/k1_err.log; exit 1; }
    tail -1 $O/k1_lb5_ab.jsonl
  done
done
for interp in nearest bilinear; do
  for pass in 1 2 3; do
    for arm in product $ARMS; do
      L=xcube-resampling_amd/lib/libxrs.so
      [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
      XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 20 --interp $interp > $O/t_${arm}_${interp}_$pass.log 2>&1 || exit $?
      echo "$arm $interp $pass $(grep 'ms per' $O/t_${arm}_${interp}_$pass.log)"
    done
  done
done
for arm in product $ARMS; do
  L=xcube-resampling_amd/lib/libxrs.so
  [ $arm = product ] || L=probe/$arm/pkg/lib/libxrs.so
  XRS_LIBRARY=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$arm -o ks -- python3 scripts/time_rectify.py --fused --reps 10 > $O/ks_$arm.log 2>&1 || exit $?
  echo "$arm nearest"; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes
done
