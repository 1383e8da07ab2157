# Round 5: what the claim's VALU issue is made of — the available counters
# (rocprofv3 --list-avail) and per-kernel instruction counts at config 4
# (VALU total / float64 by kind / transcendental, SALU, and the VALU issue
# cycles), one counter pass each.
#   bash scripts/gpu_r05_j.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05j}; mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || echo "list-avail status $?"
grep -o "SQ_INSTS_VALU[A-Z0-9_]*\|SQ_ACTIVE_INST_[A-Z]*\|SQ_INSTS_SALU\|SQ_INST_CYCLES_VALU\|SQ_INSTS_LDS\|SQ_INSTS_VMEM[A-Z_]*" $O/list_avail.txt | sort -u | head -60
timeout -k 10 150 python3 scripts/pmc_kernels.py --counters SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_INSTS_SALU,SQ_WAVES,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_LDS,SQ_INSTS_SMEM -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_a.json 2> $O/pmc_a.err; echo "a $?"; cat $O/pmc_a.json
timeout -k 10 150 python3 scripts/pmc_kernels.py --counters SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU_ADD_F32,SQ_INSTS_VALU_MUL_F32,SQ_INSTS_VALU_FMA_F32,SQ_INSTS_VALU_TRANS_F32 -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_b.json 2> $O/pmc_b.err; echo "b $?"; cat $O/pmc_b.json
timeout -k 10 150 python3 scripts/pmc_kernels.py --counters SQ_INSTS_VALU_INT32,SQ_INSTS_VALU_INT64,SQ_INSTS_VALU_CVT,SQ_INSTS_VALU_MFMA_F32,SQ_INSTS_VALU_F32_PK,SQ_ACTIVE_INST_SALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_c.json 2> $O/pmc_c.err; echo "c $?"; cat $O/pmc_c.json
true
