#!/bin/bash
# r05: the hashed 0/1 emission (tiles without a duplicated key skip the general count and
# write passes). Parity files, then tools/r05_env.sh A/B (DFP_HJ_COUNT_FREE=0 restores the
# general passes).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05h01}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_multikey.py tests/test_gpu_join_types.py} -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
RUNS=${RUNS:-"on:DFP_HJ_COUNT_FREE=1 off:DFP_HJ_COUNT_FREE=0"} CFGS=${CFGS:-"c2h c3"} BCFGS=${BCFGS:-c2h} REPS=${REPS:-2} bash tools/r05_env.sh ${1:-r05h01}
