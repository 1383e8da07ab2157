# rocprofv3 kernel stats of the config lines (scripts/bench_configs.py) and
# the band rehearsal of the multi-GPU split.   bash scripts/gpu_prof_configs.sh OUTDIR [CONFIGS]
export TMPDIR=/tmp
OUT=$1; C=${2:-1,2,3,4}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o cfg -- python3 scripts/bench_configs.py --configs $C --cpu-seconds 0.2 > $OUT/configs.jsonl 2> $OUT/configs.err || exit $?
cut -c1-300 $OUT/configs.jsonl
python3 - $OUT/prof/cfg_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Calls']:>5} {float(r['AverageNs'])/1e3:10.1f} us  {r['Name'][:150]}")
PY
timeout -k 10 300 python -u scripts/rehearse_bands.py > $OUT/bands.jsonl 2> $OUT/bands.err || exit $?
cut -c1-200 $OUT/bands.jsonl
