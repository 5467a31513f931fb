#!/bin/bash
# Iteration run: parity subset, bench lines of C2 / C2h / C3, serialized kernel stats (one MI355X).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-it6}; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
step 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${2:-parity or golden or sharded or large or smoke}" > $O/tests.log 2>&1
tail -2 $O/tests.log
for c in c2 c2h c3; do
  step 300 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['probe_ms'], d.get('build_ms'), d['roofline']['frac'])" $O/bench_$c.json $c
  step 300 rocprofv3 --kernel-trace --stats -d $O/ks_$c -o ks --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --same-stream --sync-steps --steps 5 --warmup 3 > $O/ks_$c.json 2> $O/ks_$c.err
  python3 tools/kstats.py $O/ks_$c > $O/ks_$c.txt; grep -E "sl_|hs_" $O/ks_$c.txt
done
echo "iter done"
