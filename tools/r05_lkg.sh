#!/bin/bash
# r05: dense lookup row groups (product = 4; variants 2 / 8)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05l}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
   -k "sliced or c2_full or c3_full or heavy or exponential or random_parity or explicit or probe_base" > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
for cfg in c2 c3; do
  for v in prod lkg2 lkg8; do
    L=""; [ $v != prod ] && L=tools/lib/$v.so
    DFP_HJ_LIB_VARIANT=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_${cfg}_$v -o ks --output-format csv -- \
        python3 tools/probe_one.py --config=$cfg > $O/ks_${cfg}_$v.log 2>&1 || exit $?
    python3 tools/kstats.py $O/ks_${cfg}_$v | grep -E "sl_lookup" | sed "s/^/$cfg $v /"
  done
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'], 'probe_ms', d['probe_ms'], 'frac', d['roofline']['frac'])" $O/bench_$cfg.json $cfg
done
