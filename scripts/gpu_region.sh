export TMPDIR=/tmp
O=${1:-gpurun_out/region}; shift; mkdir -p $O
timeout -k 10 300 python -u scripts/copy_variants.py "$@" > $O/copy.jsonl 2> $O/copy.err || { tail -20 $O/copy.err; exit 1; }
cat $O/copy.jsonl
