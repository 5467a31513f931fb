#!/bin/bash
# r05: settler check: spec-build / operator / multikey / parity tests, then bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05r}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_operator.py tests/test_gpu_multikey.py tests/test_gpu_multi_table.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
for cfg in c2h c2 c3; do
  for st in 1 0; do
    DFP_HJ_SETTLE=$st timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > $O/bench_${cfg}_s$st.json 2> $O/bench_${cfg}_s$st.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'], 'probe_ms', d['probe_ms'], 'build_ms', d.get('build_ms'), 'frac', d['roofline']['frac'])" $O/bench_${cfg}_s$st.json ${cfg}_settle$st
  done
done
