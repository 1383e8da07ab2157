# K1 launch-ramp diagnosis: clock probe between launches,
# then a GRBM_GUI_ACTIVE pass (effective clock per dispatch), then the bench
# line with the driver's --warmup 5.   bash scripts/gpu_ramp.sh OUTDIR
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ramp}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/ramp_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
python -c "
import json
for l in open('$OUT/probe.jsonl'):
    d=json.loads(l); print(d['pattern'], 'ms', d['ms'][:14], '...', d['ms'][-3:]); print('   GHz', d['clock_GHz'][:14], '...', d['clock_GHz'][-3:])
"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $OUT/pmc -o pmc -- python -u scripts/ramp_probe.py > $OUT/probe_pmc.jsonl 2> $OUT/probe_pmc.err || { tail -20 $OUT/probe_pmc.err; exit 1; }
timeout -k 10 300 python -u bench.py --warmup 5 --no-cpu-baseline --no-traffic > $OUT/bench_w5.json 2> $OUT/bench_w5.err || exit 1
cut -c1-300 $OUT/bench_w5.json
