#!/bin/bash
# GPU test pass: the round-4 tests first, then the whole GPU suite and smoke.
# Every GPU step under its own timeout; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04t}; mkdir -p $O
step() { local t=$1; shift; echo "== $*"; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
PT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
step 420 $PT tests/test_gpu_sharded_build.py tests/test_gpu_operator.py tests/test_gpu_tpch.py -k "budget or multi_gpu or sf300 or one_rank or native" > $O/new_tests.log 2>&1
tail -2 $O/new_tests.log
step 700 $PT tests -m gpu > $O/tests.log 2>&1
tail -2 $O/tests.log
step 60 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
