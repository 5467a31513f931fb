#!/bin/bash
# Diagnostic: partitioned-probe kernel time and L2 hit counters vs piece size (GPU box).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ppsweep
for kb in 2048 1024 512; do
  DFP_HJ_PROBE_MODE=partitioned DFP_HJ_PIECE_KB=$kb timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    -d gpurun_out/ppsweep/t_$kb -o t --output-format csv -- python3 tools/probe_one.py 1e7 > gpurun_out/ppsweep/t_$kb.log 2>&1
  DFP_HJ_PROBE_MODE=partitioned DFP_HJ_PIECE_KB=$kb timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum \
    -d gpurun_out/ppsweep/p_$kb -o p --output-format csv -- python3 tools/probe_one.py 1e7 > gpurun_out/ppsweep/p_$kb.log 2>&1
done
