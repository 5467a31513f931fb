#!/bin/bash
# r05: probe tiles of 2^14 vs 2^15 rows (DFP_HJ_SL_TILE_LOG): parity of the GPU parity suite
# with 2^15-row tiles, serialized kernel stats of the probe (probe_one), alternating bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05tl}; mkdir -p $O
TLS=${TLS:-"14 15"}
if [ -z "$SKIPTESTS" ]; then
  DFP_HJ_SL_TILE_LOG=15 timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q --timeout 300 --timeout-method thread > $O/tests_tl15.log 2>&1 || { echo "tests tl15 failed"; tail -30 $O/tests_tl15.log; exit 1; }
  echo "tl15: $(tail -1 $O/tests_tl15.log)"
fi
for cfg in ${CFGS:-c2 c3}; do
  for tl in $TLS; do
    DFP_HJ_SL_TILE_LOG=$tl timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_${cfg}_$tl -o ks --output-format csv -- \
        python3 tools/probe_one.py --config=$cfg > $O/ks_${cfg}_$tl.log 2>&1 || exit $?
    python3 tools/kstats.py $O/ks_${cfg}_$tl | grep -E "sl_|hs_" | sed "s/^/$cfg tl$tl /"
  done
done
for rep in 1 2; do
  for cfg in ${BCFGS:-c2 c3}; do
    for tl in $TLS; do
      DFP_HJ_SL_TILE_LOG=$tl timeout -k 10 300 python3 bench.py --no-cpu-baseline --config $cfg > $O/bench_${cfg}_${tl}_$rep.json 2> $O/bench_${cfg}_${tl}_$rep.err || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['probe_ms'], d['roofline']['frac'], d.get('build_ms'))" $O/bench_${cfg}_${tl}_$rep.json "$cfg tl$tl rep$rep"
    done
  done
done
