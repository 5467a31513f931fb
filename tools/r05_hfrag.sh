#!/bin/bash
# r05: hashed sliced lookup time against fragment length (P = 10^8, B = 0.5 / 1 / 2 x 10^7: fragments of 16.8 / 8.4 / 4.2 entries)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05hf}; mkdir -p $O
for B in ${BS:-5e6 1e7 2e7}; do P=1e8
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_$B -o ks --output-format csv -- \
      python3 tools/probe_one.py $B $P --mix > $O/ks_$B.log 2>&1 || exit $?
  python3 tools/kstats.py $O/ks_$B | grep -E "sl_lookup|sl_emit|hs_partition" | sed "s/^/B=$B /"
done
