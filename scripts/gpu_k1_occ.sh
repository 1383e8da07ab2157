# K1 arms (round 4): waves per SIMD forced to 5 / 6 (register caps) and the
# XCDs sweeping contiguous eighths of the item list; each arm's raster checksum
# against the product's, then bench A/B interleaved on one box.
#   bash scripts/gpu_k1_occ.sh OUTDIR   (probes: scripts/build_probe.sh)
export TMPDIR=/tmp
O=${1:-gpurun_out/k1occ}; mkdir -p $O
ARMS=${ARMS:-"base k1w5 k1w6 k1cont k1w5c"}; PASSES=${PASSES:-2}
lib() { if [ $1 = base ]; then echo xcube-resampling_amd/lib/libxrs.so; else echo probe/$1/pkg/lib/libxrs.so; fi; }
for arm in $ARMS; do
  XRS_LIBRARY=$(lib $arm) timeout -k 10 180 python -u scripts/k1_hash.py > $O/hash_$arm.txt 2> $O/hash_$arm.err || exit $?
  echo "hash $arm $(cat $O/hash_$arm.txt)"
done
B="bench.py --no-cpu-baseline --no-traffic --steps 30 --warmup 10"
for pass in $(seq 1 $PASSES); do
  for arm in $ARMS; do
    XRS_LIBRARY=$(lib $arm) timeout -k 10 300 python -u $B > $O/ab_${arm}_$pass.json 2> $O/ab_${arm}_$pass.err || exit $?
    python -c "import json; d=json.load(open('$O/ab_${arm}_$pass.json')); print('$arm', $pass, d['roofline']['kernel_ms'], d['ms_per_step'], d['f64_out']['kernel_ms'])"
  done
done
# the traffic of an arm (bench line with its two PMC passes)
if [ -n "$TRAFFIC_ARM" ]; then
  XRS_LIBRARY=$(lib $TRAFFIC_ARM) timeout -k 10 600 python -u bench.py --no-cpu-baseline --warmup 5 > $O/traffic_$TRAFFIC_ARM.json 2> $O/traffic_$TRAFFIC_ARM.err || exit $?
  cut -c1-300 $O/traffic_$TRAFFIC_ARM.json
fi
