# Memory-pipeline PMC of K1 (scripts/pmc_traffic.py: calibration + bench
# launch) for the product library and probe arms; two passes per arm.
#   bash scripts/gpu_pmc_k1_arms.sh OUTDIR ARM...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for arm in base "$@"; do
  if [ $arm = base ]; then L=xcube-resampling_amd/lib/libxrs.so; else L=probe/$arm/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -s KILL 150 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/$arm/p1 -o p1 -- python3 scripts/pmc_traffic.py > $O/$arm.p1.log 2>&1 || exit 1
  XRS_LIBRARY=$L timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/$arm/p2 -o p2 -- python3 scripts/pmc_traffic.py > $O/$arm.p2.log 2>&1 || exit 1
done
echo done
