# PMC instruction mix of the rectify kernels at config 4 (fused nearest pass of
# scripts/time_rectify.py; two passes, one counter group each; DESIGN.md §3 /
# §8 cite the result; scripts/pmc_summary.py reduces the CSVs).
#   bash scripts/pmc_rectify.sh [OUTDIR]  -> OUTDIR/{p1,p2}/*_counter_collection.csv
export TMPDIR=/tmp; O=${1:-gpurun_out/pmc4}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/p1 -o p1 -- python3 scripts/time_rectify.py --fused --reps 2 > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $O/p2 -o p2 -- python3 scripts/time_rectify.py --fused --reps 2 > $O/p2.log 2>&1 &&
for p in p1 p2; do python3 scripts/pmc_summary.py $O/$p/${p}_counter_collection.csv claim resolve ij_bboxes; done
