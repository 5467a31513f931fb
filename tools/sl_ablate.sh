#!/bin/bash
# Timing ablations of the sliced probe's emission kernel (DFP_HJ_SL_DBG; pairs are wrong
# under every nonzero value): kernel-trace per variant. usage: tools/sl_ablate.sh TAG
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for d in ${DBGS:-0 1 2 3}; do
  DFP_HJ_SL_DBG=$d DFP_HJ_PROBE_MODE=sliced timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/d$d -o s --output-format csv \
    -- python3 tools/probe_one.py > $O/d$d.log 2>&1 || { tail -20 $O/d$d.log; exit 1; }
  echo "dbg=$d"; python3 tools/kstats.py $O/d$d/s_kernel_stats.csv | grep -E "sl_"
done
