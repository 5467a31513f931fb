#!/bin/bash
# r05: the dense lookup's time against fragment length (probe keys over 2x / 1x / 4x the build range)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05i}; mkdir -p $O
for pr in 2 1 4; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_pr$pr -o ks --output-format csv -- \
      python3 tools/probe_one.py 1e7 1e8 --prange=$pr > $O/ks_pr$pr.log 2>&1 || exit $?
  python3 tools/kstats.py $O/ks_pr$pr | grep -E "sl_" | sed "s/^/prange=$pr /"
done
