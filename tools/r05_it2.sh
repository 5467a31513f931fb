#!/bin/bash
# r05: kernel stats of the sliced probe (probe_one) for the product library and optional variants
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05m}; mkdir -p $O
CFGS=${CFGS:-"c2 c3 c2h"}
VARS=${VARS:-"prod"}
TESTK=${TESTK:-"sliced or c2_full or c3_full or c2h or heavy or exponential or random_parity or explicit or probe_base or hashed"}
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "$TESTK" > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
for cfg in $CFGS; do
  for v in $VARS; do
    L=""; [ $v != prod ] && L=tools/lib/$v.so
    DFP_HJ_LIB_VARIANT=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_${cfg}_$v -o ks --output-format csv -- \
        python3 tools/probe_one.py --config=$cfg > $O/ks_${cfg}_$v.log 2>&1 || exit $?
    python3 tools/kstats.py $O/ks_${cfg}_$v | grep -E "sl_|hs_" | sed "s/^/$cfg $v /"
  done
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'], 'probe_ms', d['probe_ms'], 'build_ms', d.get('build_ms'), 'frac', d['roofline']['frac'])" $O/bench_$cfg.json $cfg
done
