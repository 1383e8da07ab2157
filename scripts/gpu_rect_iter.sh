# Rectify iteration: K4/K5/K6 parity tests, kernel stats of the config-4
# kernels in isolation, and one PMC pass of the instruction mix.
#   bash scripts/gpu_rect_iter.sh [outdir]
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ri}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_rectify_gpu.py tests/test_spatial_gpu.py -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o c4 -- python3 scripts/time_rectify.py --reps 10 > $OUT/time.log 2>&1 || exit $?
grep "ms per" $OUT/time.log
cut -d, -f1-4 $OUT/stats/c4_kernel_stats.csv | cut -c1-160 | head -8
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/p1 -o p1 -- python3 scripts/time_rectify.py --reps 2 > $OUT/p1.log 2>&1
