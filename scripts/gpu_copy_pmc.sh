# Copy-rate variants (scripts/copy_variants.py), the counter list of this
# rocprofv3, and two SQ PMC passes of K1 at config 5 (scripts/pmc_traffic.py).
#   bash scripts/gpu_copy_pmc.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/copy}; mkdir -p $O
timeout -k 10 200 python -u scripts/copy_variants.py > $O/copy.jsonl 2> $O/copy.err || { tail -20 $O/copy.err; exit 1; }
cat $O/copy.jsonl
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/p1 -o p1 -- python3 scripts/pmc_traffic.py > $O/p1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/p2 -o p2 -- python3 scripts/pmc_traffic.py > $O/p2.log 2>&1 || exit 1
echo done
