export TMPDIR=/tmp; O=gpurun_out/k1band; mkdir -p $O
timeout -k 10 400 python -u scripts/ab_reproject.py --variants 12,12@0/16,12@0/64,12@0/128,12@2/32,12@4/64 --rounds 5 > $O/ab.log 2>&1
cat $O/ab.log
