#!/bin/bash
# Round 6 GPU session driver (one MI355X via gpurun). Every GPU step under its own timeout;
# the first failure ends the script.
#   PHASE=tests   GPU tests (TESTS=<pytest args>, default the whole -m gpu suite) + smoke
#   PHASE=bench   bench lines for CFGS (default c2 c3 c2h); CPUB=1 adds C2's cpu_baseline
#   PHASE=ks      serialized kernel stats (tools/probe_one.py) per config in CFGS, for every
#                 RUNS entry "name:VAR=VAL[,VAR=VAL]" (default one run "prod:")
#   PHASE=ab      alternating bench lines per RUNS entry (REPS rounds) for CFGS
#   PHASE=pmc     FETCH_SIZE / WRITE_SIZE passes of the bench per config -> traffic_<cfg>.txt
#   PHASE=kt      rocprofv3 kernel trace of the default bench (C2)
# PHASES="tests bench" runs several in order.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06}; mkdir -p $O
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
for PH in ${PHASES:-$PHASE}; do
case $PH in
tests)
  step ${TT:-900} python3 -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  tail -2 $O/tests.log
  step 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log ;;
bench)
  for cfg in ${CFGS:-c2 c3 c2h}; do
    cb=--no-cpu-baseline; [ "$cfg" = c2 ] && [ -n "$CPUB" ] && cb=
    step 400 python3 bench.py --config $cfg $cb > $O/bench_$cfg.json 2> $O/bench_$cfg.err
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['probe_ms'], d['roofline']['frac'], d.get('build_ms'))" $O/bench_$cfg.json $cfg
  done ;;
ks)
  for cfg in ${CFGS:-c2 c3 c2h}; do
    for r in ${RUNS:-prod:}; do
      n=${r%%:*}; ev=${r#*:}
      env ${ev//,/ } timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ks_${cfg}_$n -o ks --output-format csv -- \
          python3 tools/probe_one.py --config=$cfg > $O/ks_${cfg}_$n.log 2>&1 || { echo "FAILED ks $cfg $n"; exit 1; }
      python3 tools/kstats.py $O/ks_${cfg}_$n | grep -E "sl_|hs_|frag|minmax|part" | sed "s/^/$cfg $n /"
    done
  done ;;
ab)
  for rep in $(seq 1 ${REPS:-2}); do
    for cfg in ${CFGS:-c2}; do
      for r in $RUNS; do
        n=${r%%:*}; ev=${r#*:}
        env ${ev//,/ } timeout -k 10 300 python3 bench.py --no-cpu-baseline --config $cfg > $O/ab_${cfg}_${n}_$rep.json 2> $O/ab_${cfg}_${n}_$rep.err || { echo "FAILED ab $cfg $n"; exit 1; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['probe_ms'], d['roofline']['frac'], d.get('build_ms'))" $O/ab_${cfg}_${n}_$rep.json "$cfg $n rep$rep"
      done
    done
  done ;;
pmc)
  for cfg in ${CFGS:-c2}; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      step 240 rocprofv3 --pmc $ctr -d $O/pmc_$cfg/pmc_$ctr -o pmc --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_${cfg}_$ctr.log 2>&1
    done
    python3 tools/traffic_summary.py $O/pmc_$cfg $cfg > $O/traffic_$cfg.txt
    head -30 $O/traffic_$cfg.txt
  done ;;
sq)
  # SQ counters of the sliced kernels (tools/probe_one.py), one rocprofv3 pass per counter set
  # and RUNS entry; CTRS1 / CTRS2 (<= 8 SQ counters each)
  C1=${CTRS1:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"}
  C2=${CTRS2:-"SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVES"}
  for cfg in ${CFGS:-c3}; do
    for r in ${RUNS:-prod:}; do
      n=${r%%:*}; ev=${r#*:}; i=0
      for C in "$C1" "$C2"; do
        i=$((i+1))
        env ${ev//,/ } timeout -s KILL 120 rocprofv3 --pmc $C -d $O/sq_${cfg}_${n}_$i -o pmc --output-format csv -- \
            python3 tools/probe_one.py --config=$cfg > $O/sq_${cfg}_${n}_$i.log 2>&1 || { echo "FAILED sq $cfg $n"; exit 1; }
        python3 tools/pmc_kernels.py $O/sq_${cfg}_${n}_$i "sl_lookup|hs_part|sl_emit|sl_partition" | sed "s/^/$cfg $n /"
      done
    done
  done ;;
kt)
  step 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > $O/kt_c2.json 2> $O/kt_c2.err
  python3 tools/kstats.py $O/kt_c2 > $O/kt_c2.txt; head -8 $O/kt_c2.txt ;;
esac
done
