# Round 5: config 3's kernels one by one (rocprofv3 kernel stats of the
# coarsen timing script): how much of the launch the tables kernel and the
# finish take beside K3i.
#   bash scripts/gpu_r05_ac.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/r05ac}; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- python3 scripts/time_coarsen.py > $O/ks.log 2>&1 || exit $?
tail -2 $O/ks.log
python3 scripts/kstats.py $(find $O/ks -name "*kernel_stats.csv" | head -1) affine integral finish tables
