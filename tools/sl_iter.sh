#!/bin/bash
# One iteration on the sliced probe: its parity tests, then a kernel-trace profile of the
# fused-vs-sliced sweep. usage: tools/sl_iter.sh TAG [sweep args...]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "sliced" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o s --output-format csv -- python3 tools/sliced_sweep.py ${*:-1e8 1e7} \
  > $O/sweep.log 2>&1 || { tail -30 $O/sweep.log; exit 1; }
grep -E "B=|agree" $O/sweep.log
python3 tools/kstats.py $O/s_kernel_stats.csv | grep -E "sl_|scan|probe_fused"
