# K1 work shapes through the test knobs (round 4: persistent lockstep grids
# of short items against the product's one-shot 32-row items).
#   bash scripts/gpu_k1_knob.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/k1knob}; mkdir -p $O
timeout -k 10 600 python -u scripts/k1_knob_ab.py --passes 2 > $O/knob.jsonl 2> $O/knob.err || { tail -20 $O/knob.err; exit 1; }
cut -c1-160 $O/knob.jsonl
