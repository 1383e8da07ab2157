# Round 5: what the non-separable path issues — per-kernel instruction mix of
# the config-2u kernels (xrs_transform, K1c, the fused gather) in three
# counter passes.
#   bash scripts/gpu_r05_m.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05m}; mkdir -p $O
K=transform,gather_2d,gather_proj
timeout -k 10 150 python3 scripts/pmc_kernels.py --kernels $K --counters SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_INSTS_SALU,SQ_WAVES,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES -- scripts/time_2u.py --reps 3 > $O/pmc_a.json 2> $O/pmc_a.err; echo "a $?"; cat $O/pmc_a.json
timeout -k 10 150 python3 scripts/pmc_kernels.py --kernels $K --counters SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU_ADD_F32,SQ_INSTS_VALU_MUL_F32,SQ_INSTS_VALU_FMA_F32,SQ_INSTS_VALU_TRANS_F32 -- scripts/time_2u.py --reps 3 > $O/pmc_b.json 2> $O/pmc_b.err; echo "b $?"; cat $O/pmc_b.json
timeout -k 10 150 python3 scripts/pmc_kernels.py --kernels $K --counters SQ_INSTS_VALU_INT32,SQ_INSTS_VALU_INT64,SQ_INSTS_VALU_CVT,SQ_ACTIVE_INST_ANY,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,GRBM_GUI_ACTIVE -- scripts/time_2u.py --reps 3 > $O/pmc_c.json 2> $O/pmc_c.err; echo "c $?"; cat $O/pmc_c.json
true
