#!/bin/bash
# Round 5 GPU passes at HEAD (one MI355X via gpurun). Every GPU step under its own
# timeout; the first failure ends the script.
#   PHASE=prof  PMC traffic passes of the C2 / C3 benches (FETCH_SIZE and WRITE_SIZE in
#               separate runs) -> profiles/traffic_<cfg>.json, and the kernel traces
#   PHASE=bench the whole GPU suite, smoke, the bench lines (C2 with its CPU baseline)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05close}; mkdir -p $O
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
B="python3 bench.py --no-cpu-baseline"
if [ "$PHASE" = "prof" ]; then
  for cfg in ${PMC_CFGS:-c2}; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      step 240 rocprofv3 --pmc $ctr -d $O/pmc_$cfg/pmc_$ctr -o pmc --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_${cfg}_$ctr.log 2>&1
    done
    python3 tools/traffic_summary.py $O/pmc_$cfg $cfg > $O/traffic_$cfg.txt
    head -30 $O/traffic_$cfg.txt
  done
  step 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > $O/kt_c2.json 2> $O/kt_c2.err
  python3 tools/kstats.py $O/kt_c2 > $O/kt_c2.txt; head -8 $O/kt_c2.txt
  for cfg in ${KS_CFGS:-c2 c3 c2h}; do
    step 300 rocprofv3 --kernel-trace --stats -d $O/ks_$cfg -o ks --output-format csv -- python3 bench.py --no-cpu-baseline --config $cfg --same-stream --sync-steps --steps 5 --warmup 3 > $O/ks_$cfg.json 2> $O/ks_$cfg.err
    python3 tools/kstats.py $O/ks_$cfg > $O/ks_$cfg.txt; head -6 $O/ks_$cfg.txt
  done
else
  step 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  tail -2 $O/tests.log
  step 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
  step 400 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err
  cat $O/bench_c2.json
  for cfg in c3 c2h; do
    step 300 $B --config $cfg > $O/bench_$cfg.json 2> $O/bench_$cfg.err
    cat $O/bench_$cfg.json
  done
fi
