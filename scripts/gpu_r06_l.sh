# Round 6, twelfth pass: the claim walk chosen per wave and row (compacted when
# a window of the previous row held more than 8 pixels), against every
# tile compacted (knob 1) and every tile per lane (knob 2), at config 4 and at
# finer targets (--res-div 1.25 .. 3); the rectify suite first (both walks
# forced on the forms geometries and at config-4 full size), then kernel stats.
#   bash scripts/gpu_r06_l.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06l}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "parity: $(tail -1 $O/pytest.log)"
[ $rc -eq 0 ] || { echo "pytest status $rc"; exit $rc; }
for div in 1 1.1 1.25 1.5 2 3; do
  for pass in 1 2; do
    for mode in 0 1 2; do
      timeout -k 10 180 python -u scripts/time_rectify.py --fused --reps 10 --res-div $div --compact $mode > $O/t_${div}_${mode}_$pass.log 2>&1 || exit $?
      echo "$pass $(grep 'ms per' $O/t_${div}_${mode}_$pass.log)"
    done
  done
done
for div in 1 2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$div -o ks -- python3 scripts/time_rectify.py --fused --reps 10 --res-div $div > $O/ks_$div.log 2>&1 || exit $?
  echo "product res/$div"; python3 scripts/kstats.py $(find $O/ks_$div -name "*kernel_stats.csv" | head -1) rectify
done
