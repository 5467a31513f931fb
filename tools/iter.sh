#!/bin/bash
# Iteration run on one MI355X (via gpurun): a parity subset, then bench lines and kernel
# traces of the configs named. Every GPU step under its own timeout; stops at the first
# failure.
# usage: tools/iter.sh TAG "PYTEST -k EXPR" "CONFIGS (c2 c2h c3 radix bcast)" [trace]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; K=$2; CFGS=$3; TRACE=$4
O=gpurun_out/$TAG; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
if [ -n "$K" ]; then
  step 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
  tail -2 $O/tests.log
fi
for c in $CFGS; do
  case $c in
    radix) A="--force-dist --plan radix --steps 20 --warmup 5" ;;
    bcast) A="--force-dist --plan broadcast --steps 20 --warmup 5" ;;
    sharded) A="--force-dist --plan sharded --steps 20 --warmup 5" ;;
    *) A="--config $c" ;;
  esac
  step 300 python3 bench.py $A --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['probe_ms'], d.get('build_ms'), d['roofline']['frac'])" $O/bench_$c.json $c
  if [ -n "$TRACE" ]; then
    step 300 rocprofv3 --kernel-trace --stats -d $O/kt_$c -o kt --output-format csv -- python3 bench.py $A --no-cpu-baseline > $O/kt_$c.json 2> $O/kt_$c.err
    python3 tools/kstats.py $O/kt_$c | head -12
  fi
done
echo "iter $TAG done"
