# One PMC pass (wave cycles / waits / instruction counts) of time_rectify.py
# for the product library and each probe named on the command line.
#   bash scripts/gpu_probe_pmc.sh OUT probe1 probe2 ...
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for p in product "$@"; do
  if [ $p = product ]; then L=xcube_resampling_amd/lib/libxrs.so; else L=probe/$p/pkg/lib/libxrs.so; fi
  XRS_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $O/$p -o p -- python3 scripts/time_rectify.py --reps 2 > $O/$p.log 2>&1 || exit $?
done
