# Round 6, second pass: the whole GPU suite on the product (round-5 claim,
# K4 DPP extremes, stream-synchronising unregister, two-step projection
# decisions, config 5 on all tiles); rectify arms (resolve bands dealt to the
# XCDs in runs, K4 next-block prefetch at 16 / 8 rows) for parity and
# interleaved timing with kernel stats; PMC read / write traffic per rectify
# kernel; the config-4 line with the fused pipeline's own kernel times.
#   bash scripts/gpu_r06_b.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06b}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --durations 8 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -12 $O/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest status $rc"; exit $rc; }
ARMS="rxcd k4pf k4pf8"
for arm in $ARMS; do
  XRS_LIBRARY=probe/$arm/pkg/lib/libxrs.so timeout -k 10 300 python -u -m pytest tests/test_rectify_gpu.py -m gpu -q -x -k "config4_full or fused_resolve or k4_ or triangle_keys or filled_claim" --timeout 200 --timeout-method thread > $O/pytest_$arm.log 2>&1; rc=$?
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
  echo $arm; python3 scripts/kstats.py $(find $O/ks_$arm -name "*kernel_stats.csv" | head -1) claim resolve bboxes tiles
done
timeout -k 10 200 python -u scripts/pmc_kernels.py --counters TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum --kernels claim,resolve,ij_bboxes -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_rd.json 2> $O/pmc_rd.err || exit $?
timeout -k 10 200 python -u scripts/pmc_kernels.py --counters TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum --kernels claim,resolve,ij_bboxes -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_wr.json 2> $O/pmc_wr.err || exit $?
cat $O/pmc_rd.json $O/pmc_wr.json | cut -c1-400
timeout -k 10 600 python -u scripts/bench_configs.py --configs 4 --cpu-seconds 3 > $O/config4.jsonl 2> $O/config4.err || { tail -20 $O/config4.err; exit 1; }
cut -c1-400 $O/config4.jsonl
