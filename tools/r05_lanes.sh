#!/bin/bash
# r05: A/B of the dense lookup variants (DFP_HJ_SL_LANES = lanes per fragment, _U = positions in flight)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05h}; mkdir -p $O
VARIANTS=${VARIANTS:-"0:4 4:4 8:4 16:2 16:1 32:1 32:2 64:1"}
# parity of the new kernel first (sliced probes, C2/C3 full size)
DFP_HJ_SL_LANES=4 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
   -k "sliced or c2_full or c3_full or heavy or exponential or random_parity or explicit or probe_base" > $O/tests_l4.log 2>&1 || exit $?
tail -1 $O/tests_l4.log
for cfg in c2 c3; do
  for v in $VARIANTS; do
    L=${v%%:*}; U=${v##*:}
    DFP_HJ_SL_LANES=$L DFP_HJ_SL_LANES_U=$U timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_${cfg}_$L_$U -o ks --output-format csv -- \
        python3 tools/probe_one.py --config=$cfg > $O/ks_${cfg}_${L}_$U.log 2>&1 || exit $?
    python3 tools/kstats.py $O/ks_${cfg}_$L_$U | grep -E "sl_lookup" | sed "s/^/$cfg L=$L U=$U /"
  done
done
