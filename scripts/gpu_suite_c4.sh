# GPU suite, config-4 kernel stats and the config-4 bench line.
export TMPDIR=/tmp
OUT=${1:-gpurun_out/s4}
mkdir -p $OUT
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest ended with status $rc"; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rect -o c4 -- python3 scripts/time_rectify.py --reps 10 --fused > $OUT/rect_time.log 2>&1 || exit $?
grep "ms per" $OUT/rect_time.log
cut -d, -f1-4 $OUT/rect/c4_kernel_stats.csv | cut -c1-160 | head -5
timeout -k 10 600 python -u scripts/bench_configs.py --configs 4 --cpu-seconds 8 > $OUT/configs4.jsonl 2> $OUT/configs4.err || exit $?
cut -c1-300 $OUT/configs4.jsonl
for pass in 1 2; do
  for arm in product rg8 rg64; do
    if [ $arm = product ]; then L=""; else L=$PWD/probe/$arm/pkg/lib/libxrs.so; fi
    XRS_LIBRARY=$L timeout -k 10 120 python -u scripts/time_rectify.py --reps 20 --fused >> $OUT/rg_ab.log 2>&1 || exit $?
  done
done
grep "ms per" $OUT/rg_ab.log
