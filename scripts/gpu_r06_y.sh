# Round 6, end: the instruction mix of the final config-4 pipeline (the same
# counter passes as round 5's gpu_r05_j.sh, for the before / after of VERDICT
# r05 item 1), plus a wait pass.
#   bash scripts/gpu_r06_y.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r06y}; mkdir -p $O
timeout -k 10 150 python3 scripts/pmc_kernels.py --counters SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_INSTS_SALU,SQ_WAVES,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_LDS,SQ_INSTS_SMEM -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_a.json 2> $O/pmc_a.err || { tail $O/pmc_a.err; exit 1; }
echo a; cat $O/pmc_a.json
timeout -k 10 150 python3 scripts/pmc_kernels.py --counters SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU_ADD_F32,SQ_INSTS_VALU_MUL_F32,SQ_INSTS_VALU_FMA_F32,SQ_INSTS_VALU_TRANS_F32 -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_b.json 2> $O/pmc_b.err || { tail $O/pmc_b.err; exit 1; }
echo b; cat $O/pmc_b.json
timeout -k 10 150 python3 scripts/pmc_kernels.py --counters SQ_INSTS_VALU_INT32,SQ_INSTS_VALU_INT64,SQ_INSTS_VALU_CVT,SQ_INSTS_VALU_MFMA_F32,SQ_INSTS_VALU_F32_PK,SQ_ACTIVE_INST_SALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_c.json 2> $O/pmc_c.err || { tail $O/pmc_c.err; exit 1; }
echo c; cat $O/pmc_c.json
timeout -k 10 150 python3 scripts/pmc_kernels.py --counters SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_WAVE_CYCLES -- scripts/time_rectify.py --fused --reps 3 > $O/pmc_d.json 2> $O/pmc_d.err || { tail $O/pmc_d.err; exit 1; }
echo d; cat $O/pmc_d.json
