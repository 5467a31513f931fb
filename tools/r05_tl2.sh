#!/bin/bash
# r05: probe tiles of 2^14 vs 2^15 rows, with variant libraries (tools/lib/<v>.so).
# RUNS="tl:variant ..." (variant prod = the in-tree library)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05tl2}; mkdir -p $O
RUNS=${RUNS:-"14:prod 15:prod"}
if [ -z "$SKIPTESTS" ]; then
  DFP_HJ_SL_TILE_LOG=15 timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q --timeout 300 --timeout-method thread > $O/tests_tl15.log 2>&1 || { echo "tests tl15 failed"; tail -30 $O/tests_tl15.log; exit 1; }
  echo "tl15: $(tail -1 $O/tests_tl15.log)"
fi
for cfg in ${CFGS:-c2 c3}; do
  for r in $RUNS; do
    tl=${r%%:*}; v=${r#*:}; L=""; [ $v != prod ] && L=tools/lib/$v.so
    DFP_HJ_LIB_VARIANT=$L DFP_HJ_SL_TILE_LOG=$tl timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_${cfg}_${tl}_$v -o ks --output-format csv -- \
        python3 tools/probe_one.py --config=$cfg > $O/ks_${cfg}_${tl}_$v.log 2>&1 || exit $?
    python3 tools/kstats.py $O/ks_${cfg}_${tl}_$v | grep -E "sl_|hs_" | sed "s/^/$cfg tl$tl $v /"
  done
done
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${BCFGS:-c2 c3}; do
    BR=${BRUNS:-$RUNS}; [ "$cfg" = c2h ] && BR=${HRUNS:-$BR}
    for r in $BR; do
      tl=${r%%:*}; v=${r#*:}; L=""; [ $v != prod ] && L=$PWD/tools/lib/$v.so
      DFP_HJ_LIB=$L DFP_HJ_SL_TILE_LOG=$tl timeout -k 10 300 python3 bench.py --no-cpu-baseline --config $cfg > $O/bench_${cfg}_${tl}_${v}_$rep.json 2> $O/bench_${cfg}_${tl}_${v}_$rep.err || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['probe_ms'], d['roofline']['frac'], d.get('build_ms'))" $O/bench_${cfg}_${tl}_${v}_$rep.json "$cfg tl$tl $v rep$rep"
    done
  done
done
