#!/bin/bash
# r05: C2h probe kernels against the hashed table's load factor (DFP_HJ_LOAD_FACTOR)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05hlf}; mkdir -p $O
for LF in ${LFS:-0.5 0.6 0.7}; do
  DFP_HJ_LOAD_FACTOR=$LF timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_$LF -o ks --output-format csv -- \
      python3 tools/probe_one.py --config=c2h > $O/ks_$LF.log 2>&1 || exit $?
  python3 tools/kstats.py $O/ks_$LF | grep -E "sl_lookup|sl_emit|hs_partition|hashed_frag" | sed "s/^/lf=$LF /"
done
