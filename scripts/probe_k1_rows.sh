# K1 A/B: default (12) vs two-phase row loads (25) and the no-ceil-row timing
# probe (92, wrong values), 40960^2 and 8192^2, plus nearest for reference.
export TMPDIR=/tmp; O=gpurun_out/k1probe2; mkdir -p $O
timeout -k 10 400 python -u scripts/ab_reproject.py --variants 12,28 --rounds 5 > $O/ab.log 2>&1
cat $O/ab.log
timeout -k 10 300 python -u scripts/ab_reproject.py --size 8192 --variants 12,28 --rounds 5 > $O/ab8k.log 2>&1
cat $O/ab8k.log
timeout -k 10 300 python -u scripts/ab_reproject.py --variants 12 --interp nearest --rounds 3 > $O/abn.log 2>&1
cat $O/abn.log
