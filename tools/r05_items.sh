#!/bin/bash
# r05: sliced probe of a rank's share at N = 2 / 4 / 8 (P = 5e7 / 2.5e7 / 1.25e7, B = 1e7) against the
# lookup's item target (DFP_HJ_SLICED_ITEMS)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05q}; mkdir -p $O
for P in 1.25e7 2.5e7 5e7; do
  for it in 768 512 384 306 1024; do
    DFP_HJ_SLICED_ITEMS=$it timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_${P}_$it -o ks --output-format csv -- \
        python3 tools/probe_one.py 1e7 $P > $O/ks_${P}_$it.log 2>&1 || exit $?
    python3 tools/kstats.py $O/ks_${P}_$it | grep -E "sl_lookup|sl_emit|sl_partition" | sed "s/^/P=$P items=$it /"
  done
done
