export TMPDIR=/tmp; O=gpurun_out/k1probe; mkdir -p $O
timeout -k 10 400 python -u scripts/ab_reproject.py --variants 12,91,90 --rounds 5 > $O/ab.log 2>&1
cat $O/ab.log
timeout -k 10 300 python -u scripts/ab_reproject.py --variants 12 --interp nearest --rounds 3 > $O/abn.log 2>&1
cat $O/abn.log
