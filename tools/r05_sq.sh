#!/bin/bash
# r05: SQ wave-state counters of the sliced probe kernels (one pass each config)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05sq}; mkdir -p $O
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"}
for cfg in ${CFGS:-c2 c2h}; do
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $O/pmc_$cfg -o pmc --output-format csv -- \
      python3 tools/probe_one.py --config=$cfg > $O/pmc_$cfg.log 2>&1 || { echo "pmc $cfg failed"; exit 1; }
  python3 tools/pmc_kernels.py $O/pmc_$cfg "sl_lookup|hs_part|sl_emit|sl_partition" | sed "s/^/$cfg /"
done
