# DRAM-side queue counters of K1 under the product deal and the XCD-contiguous
# probe (scripts/build_probe.sh k1cont ...): read / write requests and their
# in-flight levels (average latency in cycles = LEVEL / requests).  PMC="..."
# replaces the counter list (e.g. the SQ side: wave cycles, vmem levels).
#   bash scripts/gpu_k1_level.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/k1level}; mkdir -p $O
PMC=${PMC:-"TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum"}
for arm in base k1cont; do
  if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $O/$arm -o lv -- python3 scripts/k1_pad_ab.py --steps 3 --tag $arm > $O/$arm.log 2>&1 || { tail -5 $O/$arm.log; exit 1; }
  tail -1 $O/$arm.log
done
python3 - "$O" <<'EOF'
import csv, glob, sys, collections
o = sys.argv[1]
for arm in ("base", "k1cont"):
    f = glob.glob(f"{o}/{arm}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "gather_separable" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    rd = m.get("TCC_EA0_RDREQ_LEVEL_sum", 0) / max(m.get("TCC_EA0_RDREQ_sum", 1), 1)
    wr = m.get("TCC_EA0_WRREQ_LEVEL_sum", 0) / max(m.get("TCC_EA0_WRREQ_sum", 1), 1)
    extra = {}
    if "SQ_INSTS_VMEM_sum" in m or "SQ_INSTS_VMEM" in m:
        iv = m.get("SQ_INSTS_VMEM_sum", m.get("SQ_INSTS_VMEM", 1))
        lv = m.get("SQ_INST_LEVEL_VMEM_sum", m.get("SQ_INST_LEVEL_VMEM", 0))
        extra["vmem_latency_cycles"] = round(lv / max(iv, 1), 1)
    print(arm, {k: round(v) for k, v in m.items()}, "read latency cycles", round(rd, 1),
          "write latency cycles", round(wr, 1), extra)
EOF
