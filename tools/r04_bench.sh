#!/bin/bash
# Round 4 bench pass: parity tests of the sliced probe, then C2 / C3 / C2h bench lines with
# the count-free emission on and off (alternating), and serialized kernel stats of C2 and C3.
# OUT names the gpurun_out subdirectory. Every GPU step under its own timeout.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04b}; mkdir -p $O
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
PT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
if [ -z "$NOTEST" ]; then
  step 400 $PT tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_join_types.py > $O/tests.log 2>&1
  tail -1 $O/tests.log
fi
B="python3 bench.py --no-cpu-baseline"
for cfg in ${CFGS:-c2 c3}; do
  for v in 1 0 1 0; do
    DFP_HJ_COUNT_FREE=$v step 200 $B --config $cfg > $O/bench_${cfg}_cf$v.json 2> $O/bench_${cfg}_cf$v.err
    echo "$cfg cf=$v $(python3 -c "import json,sys; d=json.load(open('$O/bench_${cfg}_cf$v.json')); print(d['value'], d['ms_per_step'], d.get('probe_ms'), d['roofline']['frac'])")"
  done
done
if [ -n "$KSTATS" ]; then
  for cfg in $KSTATS; do
    step 300 rocprofv3 --kernel-trace --stats -d $O/ks_$cfg -o ks --output-format csv -- python3 bench.py --no-cpu-baseline --config $cfg --same-stream --sync-steps --steps 5 --warmup 3 > $O/ks_$cfg.json 2> $O/ks_$cfg.err
    python3 tools/kstats.py $O/ks_$cfg | head -14
  done
fi
