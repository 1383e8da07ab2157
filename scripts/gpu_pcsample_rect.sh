# PC sampling of the config-4 rectify pass (fused nearest; claim + resolve):
# where the claim's issue slots go, by instruction.  host_trap sampling at a
# time interval; the CSV holds the sampled PCs (code-object offsets, with the
# instruction text when rocprofv3 decodes it).
#   bash scripts/gpu_pcsample_rect.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/pcs}; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --kernel-trace --output-format csv -d $O/p -o p -- python3 scripts/time_rectify.py --fused --reps 6 > $O/p.log 2>&1; rc=$?
tail -5 $O/p.log
ls -la $O/p 2>/dev/null | head
exit $rc
