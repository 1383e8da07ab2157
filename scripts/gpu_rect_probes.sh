# Rectify kernel stats for the product library and probe builds (probe/<name>).
#   bash scripts/gpu_rect_probes.sh OUTDIR ARM [ARM ...]
export TMPDIR=/tmp
OUT=$1; shift; mkdir -p $OUT
for arm in base "$@"; do
  if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$arm -o c4 -- python3 scripts/time_rectify.py --reps 10 > $OUT/$arm.log 2>&1 || exit $?
  echo "== $arm: $(grep 'ms per' $OUT/$arm.log)"
  python3 - $OUT/$arm/c4_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "xrs::" in r["Name"]:
        print(f"   {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
PY
done
