#!/bin/bash
# r05: hashed lookup variants (tools/lib/<v>.so): parity of the hashed tests with each
# variant library, then serialized kernel stats of the C2h probe (probe_one)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05hs}; mkdir -p $O
VARS=${VARS:-"prod hs2"}
TESTK=${TESTK:-"hashed or c2h or sliced"}
for v in $VARS; do
  [ $v = prod ] && continue
  [ -n "$SKIPTESTS" ] && continue
  DFP_HJ_LIB=tools/lib/$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "$TESTK" > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
for cfg in ${CFGS:-c2h}; do
  for v in $VARS; do
    L=""; [ $v != prod ] && L=tools/lib/$v.so
    DFP_HJ_LIB_VARIANT=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_${cfg}_$v -o ks --output-format csv -- \
        python3 tools/probe_one.py --config=$cfg > $O/ks_${cfg}_$v.log 2>&1 || exit $?
    python3 tools/kstats.py $O/ks_${cfg}_$v | grep -E "sl_|hs_" | sed "s/^/$cfg $v /"
  done
done
# PMC: LDS bank conflicts / LDS-array cycles / VALU per kernel (one counter group per run)
for v in ${PMCVARS:-}; do
  L=""; [ $v != prod ] && L=tools/lib/$v.so
  DFP_HJ_LIB_VARIANT=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_$v -o pmc --output-format csv -- \
      python3 tools/probe_one.py --config=c2h > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 tools/pmc_kernels.py $O/pmc_$v "sl_lookup|hs_part|sl_emit" | sed "s/^/pmc $v /"
done
