# Config-4 bench lines (fused vs unfused, nearest / bilinear), then the claim
# attribution arms.   bash scripts/gpu_c4_attr.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
timeout -k 10 400 python -u scripts/bench_configs.py --configs 4 --cpu-seconds 1 > $O/c4.jsonl 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
python3 -c "import json; [print(d['workload'][:18], d['ms_per_step'], d['k5_ms'], d['k6_ms'], d['unfused_ms']) for d in map(json.loads, open('$O/c4.jsonl'))]"
bash scripts/gpu_claim_attr.sh $O/attr "$@"
