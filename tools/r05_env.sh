#!/bin/bash
# r05: A/B of environment settings. RUNS="name:VAR=VAL[,VAR=VAL] ...": serialized kernel stats
# of tools/probe_one.py per config (CFGS), then alternating bench lines (BCFGS, REPS rounds)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05env}; mkdir -p $O
for cfg in ${CFGS:-c2h}; do
  for r in $RUNS; do
    n=${r%%:*}; ev=${r#*:}
    env ${ev//,/ } timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_${cfg}_$n -o ks --output-format csv -- \
        python3 tools/probe_one.py --config=$cfg > $O/ks_${cfg}_$n.log 2>&1 || exit $?
    python3 tools/kstats.py $O/ks_${cfg}_$n | grep -E "sl_|hs_|frag|minmax" | sed "s/^/$cfg $n /"
  done
done
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${BCFGS:-c2h}; do
    for r in $RUNS; do
      n=${r%%:*}; ev=${r#*:}
      env ${ev//,/ } timeout -k 10 300 python3 bench.py --no-cpu-baseline --config $cfg > $O/bench_${cfg}_${n}_$rep.json 2> $O/bench_${cfg}_${n}_$rep.err || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['probe_ms'], d['roofline']['frac'], d.get('build_ms'))" $O/bench_${cfg}_${n}_$rep.json "$cfg $n rep$rep"
    done
  done
done
