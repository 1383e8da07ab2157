# K4 attribution: config-4 kernel timing with probe arms that skip the tile
# search or the wave merge (wrong values; timing only).   bash scripts/gpu_k4_attr.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for arm in base "$@"; do
  if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${arm} -o c4 -- python3 scripts/time_rectify.py --reps 20 > $O/${arm}.log 2>&1 || exit 1
  echo "$arm"; python3 scripts/kstats.py $O/${arm}/c4_kernel_stats.csv bboxes
  XRS_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d $O/${arm}_p -o p -- python3 scripts/time_rectify.py --reps 2 > $O/${arm}_p.log 2>&1 || exit 1
  python3 - $O/${arm}_p/p_counter_collection.csv <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "bboxes" in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
d = list(acc.values())[-1]
print("  K4 PMC", {k: int(v) for k, v in sorted(d.items())})
PY
done
