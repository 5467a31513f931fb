#!/bin/bash
# The last GPU check of the round at HEAD: the whole GPU suite, smoke, the C2 bench line with
# its CPU baseline and its kernel trace (one MI355X via gpurun).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/closing; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
step 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
step 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
step 400 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err
step 300 python3 bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err
step 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > $O/kt_c2.json 2> $O/kt_c2.err
step 300 rocprofv3 --kernel-trace --stats -d $O/ks_c2 -o ks --output-format csv -- python3 bench.py --no-cpu-baseline --same-stream --sync-steps --steps 5 --warmup 3 > $O/ks_c2.json 2> $O/ks_c2.err
cat $O/bench_c2.json
