export TMPDIR=/tmp
bash scripts/gpu_rect_iter.sh gpurun_out/ri2 || exit $?
XRS_LIBRARY=probe/res8/pkg/lib/libxrs.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ri2/res8 -o c4 -- python3 scripts/time_rectify.py --reps 10 > gpurun_out/ri2/res8.log 2>&1 || exit $?
grep "ms per" gpurun_out/ri2/res8.log
cut -d, -f1-4 gpurun_out/ri2/res8/c4_kernel_stats.csv | cut -c1-160 | head -6
