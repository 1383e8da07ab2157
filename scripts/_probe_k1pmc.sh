export TMPDIR=/tmp; mkdir -p gpurun_out/k1pmc
rocprofv3 -L > gpurun_out/k1pmc/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/k1pmc -o sq -- python scripts/probe_k1.py > gpurun_out/k1pmc/sq.log 2>&1
