#!/bin/bash
# r05: hs_partition32's rank phase with 1 / 2 / 8 groups of 4 rows per scheduling region
# (tools/lib/rg2.so, rg8.so: DFP_HS32_RG). Hashed parity file with each variant, then
# tools/r05_env.sh A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05rg}; mkdir -p $O
for v in rg2 rg8; do
  DFP_HJ_LIB=tools/lib/$v.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "hashed or c2h" -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $O/tests_$v.log)"
done
RUNS="prod:DFP_HJ_SL_TAIL=1 rg2:DFP_HJ_LIB_VARIANT=tools/lib/rg2.so,DFP_HJ_LIB=tools/lib/rg2.so rg8:DFP_HJ_LIB_VARIANT=tools/lib/rg8.so,DFP_HJ_LIB=tools/lib/rg8.so" CFGS=c2h BCFGS=c2h REPS=2 bash tools/r05_env.sh ${1:-r05rg}
