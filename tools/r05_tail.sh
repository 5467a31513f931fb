#!/bin/bash
# r05: (1) the lookup's tail split chosen by the least tail-round time (C2h: 162 tail slices
# in thirds; DFP_HJ_SL_TAIL=0: the even split); (2) the lookup's per-block tile-count atomic
# issued behind the next block's entry loads (tools/lib/nodefer.so: DFP_LK_DEFER_ADD=0).
# Parity files, then tools/r05_env.sh A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05tail}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_multikey.py} -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
V=tools/lib/nodefer.so
RUNS=${RUNS:-"prod:DFP_HJ_SL_TAIL=1 tail0:DFP_HJ_SL_TAIL=0 nodefer:DFP_HJ_LIB_VARIANT=$V,DFP_HJ_LIB=$V"} CFGS=${CFGS:-"c2h c3 c2"} BCFGS=${BCFGS:-"c2h c3"} REPS=${REPS:-2} bash tools/r05_env.sh ${1:-r05tail}
