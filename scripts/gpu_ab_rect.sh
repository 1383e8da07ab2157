# Config-4 rectify A/B of the product library against probe arms, fused
# (K6 in the resolve pass) and unfused: kernel stats under rocprofv3.
#   bash scripts/gpu_ab_rect.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for arm in "$@"; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_$arm.log 2>&1 || { tail -20 $O/pytest_$arm.log; exit 1; }
  echo "$arm: $(tail -1 $O/pytest_$arm.log)"
done
for pass in 1 2; do
  for arm in base "$@"; do
    if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
    for X in "" --fused; do
      N=${arm}${X:+_fused}_$pass
      XRS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$N -o c4 -- python3 scripts/time_rectify.py --reps 20 $X > $O/$N.log 2>&1 || exit 1
      echo "$N $(grep 'ms per' $O/$N.log)"
      python3 scripts/kstats.py $O/$N/c4_kernel_stats.csv bboxes claim resolve rectify_var tiles
    done
  done
done
