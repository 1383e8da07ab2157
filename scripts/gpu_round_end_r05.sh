# Round-5 end check of the tree: the whole GPU suite, smoke, the bench line
# (driver settings, with its PMC traffic passes), the rocprofv3 kernel stats
# of the bench command, the K2 A/B (single chunk back on the per-slice
# kernel), then the secondary config lines and the band rehearsal.
#   bash scripts/gpu_round_end_r05.sh OUTDIR
export TMPDIR=/tmp
OUT=${1:-gpurun_out/end5}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest ended with status $rc"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 1 --warmup 5 --steps 20 > $OUT/bench_w5.json 2> $OUT/bench_w5.err || exit $?
cut -c1-300 $OUT/bench_w5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-traffic --no-f64 --warmup 5 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit $?
cut -c1-200 $OUT/bench_prof.json
for pass in 1 2; do
  for arm in base k2old; do
    L=xcube-resampling_amd/lib/libxrs.so
    [ $arm = base ] || L=probe/$arm/pkg/lib/libxrs.so
    XRS_LIBRARY=$L timeout -k 10 180 python -u scripts/time_affine.py --tag $arm >> $OUT/k2_ab.jsonl 2> $OUT/k2_ab_$arm.err || exit $?
    tail -1 $OUT/k2_ab.jsonl
  done
done
timeout -k 10 900 python -u scripts/bench_configs.py --configs 1,2,2u,3,4 --cpu-seconds 6 > $OUT/configs.jsonl 2> $OUT/configs.err || { tail -20 $OUT/configs.err; exit 1; }
cut -c1-160 $OUT/configs.jsonl
timeout -k 10 300 python -u scripts/rehearse_bands.py > $OUT/bands.jsonl 2> $OUT/bands.err || exit $?
cut -c1-200 $OUT/bands.jsonl
