# Full GPU suite (per-test timeout), then optional K1 A/B arms and a --warmup 5 bench.
#   bash scripts/gpu_suite3.sh OUTDIR [ARM...]
export TMPDIR=/tmp
O=${1:-gpurun_out/suite}; shift; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
fi
if [ $# -gt 0 ]; then
  B="bench.py --no-cpu-baseline --no-traffic --steps 30 --warmup 30"
  for pass in 1 2; do
    for arm in base "$@"; do
      if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
      XRS_LIBRARY=$L timeout -k 10 300 python -u $B > $O/ab_${arm}_$pass.json 2> $O/ab_${arm}_$pass.err || exit 1
      python -c "import json; d=json.load(open('$O/ab_${arm}_$pass.json')); print('$arm', $pass, d['roofline']['kernel_ms'], d['ms_per_step'], d['f64_out']['kernel_ms'], d['roofline']['copy_GBs'])"
    done
  done
fi
timeout -k 10 300 python -u bench.py --warmup 5 --no-traffic --cpu-seconds 4 > $O/bench_w5.json 2> $O/bench_w5.err || exit 1
python -c "import json; d=json.load(open('$O/bench_w5.json')); print(d['ms_per_step'], d['roofline'], d['clock_GHz'], d['cpu_baseline']['threads_sweep'])"
