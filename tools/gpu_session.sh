#!/bin/bash
# One GPU-box session: parity tests, the bench line, its rocprofv3 kernel-trace summary,
# and HBM traffic counters (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md
# "rocprofv3 PMC slots"), plus the gather microbenchmark under FETCH_SIZE to calibrate what
# the counter reports for random 16-/64-byte line accesses.
# usage: tools/gpu_session.sh TAG [tests|bench|prof|pmc|cal ...]   (default: all)
set -o pipefail
TAG=${1:-r01}; shift
STEPS=${*:-tests bench prof pmc}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
run() { echo "== $*" >&2; "$@"; }
for s in $STEPS; do
  case $s in
    tests)
      run timeout -k 10 900 python3 -m pytest tests -m gpu -x -q --timeout 300 > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
      tail -3 $O/tests.log ;;
    bench)
      run timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
      cat $O/bench.json ;;
    prof)
      run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o bench --output-format csv \
        -- python3 bench.py > $O/prof_bench.json 2> $O/prof_bench.err || { tail -30 $O/prof_bench.err; exit 1; }
      cat $O/prof_bench.json ;;
    pmc)
      # HBM traffic counters of the bench config $CFG (default c2), one counter per pass
      CFG=${CFG:-c2}
      for c in FETCH_SIZE WRITE_SIZE; do
        run timeout -k 10 400 rocprofv3 --pmc $c -d $O/$CFG/pmc_$c -o pmc --output-format csv \
          -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_${CFG}_$c.json \
          2> $O/pmc_${CFG}_$c.err || { tail -30 $O/pmc_${CFG}_$c.err; exit 1; }
      done ;;
    cal)
      run timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/cal -o cal --output-format csv \
        -- tools/ubench_gather > $O/cal.log 2> $O/cal.err || { tail -30 $O/cal.err; exit 1; }
      cat $O/cal.log ;;
    modes)
      # probe strategies side by side: one build + 5 probes each, kernel trace
      for m in fused two-pass partitioned; do
        export DFP_HJ_PROBE_MODE=$m
        run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mode_$m -o m \
          --output-format csv -- python3 tools/probe_one.py > $O/mode_$m.log 2>&1 || { tail -30 $O/mode_$m.log; exit 1; }
        unset DFP_HJ_PROBE_MODE
        tail -1 $O/mode_$m.log
      done ;;
    nt)
      # fused probe with nontemporal key loads (1) / pair stores (2)
      for v in 0 1 2 3; do
        export DFP_HJ_NT=$v
        run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/nt_$v -o m \
          --output-format csv -- python3 tools/probe_one.py > $O/nt_$v.log 2>&1 || { tail -30 $O/nt_$v.log; exit 1; }
        unset DFP_HJ_NT
      done ;;
    lf)
      # table load factor vs build / probe time
      for v in ${LFS:-0.35 0.42 0.5}; do
        export DFP_HJ_LOAD_FACTOR=$v
        run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lf_$v -o m \
          --output-format csv -- python3 tools/probe_one.py > $O/lf_$v.log 2>&1 || { tail -30 $O/lf_$v.log; exit 1; }
        unset DFP_HJ_LOAD_FACTOR
      done ;;
    c3|c2h)
      run timeout -k 10 400 python3 bench.py --config $s --no-cpu-baseline > $O/bench_$s.json 2> $O/bench_$s.err \
        || { tail -30 $O/bench_$s.err; exit 1; }
      cat $O/bench_$s.json ;;
    ablc2h)
      # hashed sliced probe ablations (DFP_HJ_SL_DBG bits, wrong pairs but in-range refs):
      # 4 no bucket lookup; per-kernel times of one build + 5 probes
      for d in 4; do
        DFP_HJ_SL_DBG=$d run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/abl$d -o kp --output-format csv \
          -- python3 tools/probe_one.py 1e7 1e8 --mix > $O/abl$d.log 2>&1 || { tail -30 $O/abl$d.log; exit 1; }
        python3 tools/kstats.py $O/abl$d | grep -E "lookup|partition|emit"
      done
      # hashed table load factor (keys per slot) vs the sliced probe
      for lf in ${LFS:-0.5 0.7 0.8}; do
        DFP_HJ_LOAD_FACTOR=$lf run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lf$lf -o kp \
          --output-format csv -- python3 tools/probe_one.py 1e7 1e8 --mix > $O/lf$lf.log 2>&1 || { tail -30 $O/lf$lf.log; exit 1; }
        echo "lf $lf: $(tail -1 $O/lf$lf.log)"
        python3 tools/kstats.py $O/lf$lf | grep -E "lookup|partition|emit|chunk_build|transpose"
      done ;;
    emitwgs)
      # persistent emission grid (workgroups per CU) vs one workgroup per tile (1000)
      for v in 2 1000; do
        DFP_HJ_SL_EMIT_WGS=$v run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ew$v -o kp --output-format csv \
          -- python3 tools/probe_one.py > $O/ew$v.log 2>&1 || { tail -30 $O/ew$v.log; exit 1; }
        echo "emit wgs $v"; python3 tools/kstats.py $O/ew$v | grep -E "sl_"
      done ;;
    kpc2h|kpc3)
      # per-kernel times of the bench config (serialized steps), kernel trace
      c=${s#kp}
      run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$s -o kp --output-format csv \
        -- python3 bench.py --config $c --no-cpu-baseline --same-stream --sync-steps --steps 5 --warmup 3 \
        > $O/$s.json 2> $O/$s.err || { tail -30 $O/$s.err; exit 1; }
      python3 tools/kstats.py $O/$s ;;
    dist)
      for pl in broadcast radix; do
        run timeout -k 10 400 python3 bench.py --force-dist --plan $pl --no-cpu-baseline --steps 5 > $O/bench_dist_$pl.json \
          2> $O/bench_dist_$pl.err || { tail -30 $O/bench_dist_$pl.err; exit 1; }
        cat $O/bench_dist_$pl.json
      done
      run timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_trun.json \
        2> $O/bench_trun.err || { tail -30 $O/bench_trun.err; exit 1; }
      cat $O/bench_trun.json ;;
    prio)
      # HIP stream priorities of the pipelined single-GPU bench (probe high / build low)
      python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
      for pr in none probe-high build-low none probe-high; do
        run timeout -k 10 300 python3 bench.py --config ${CFG:-c2} --no-cpu-baseline --stream-priority $pr \
          > $O/prio_$pr.json 2> $O/prio_$pr.err || { tail -30 $O/prio_$pr.err; exit 1; }
        echo "$pr: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['probe_ms'], d['probe_ms_in_step'], d['build_ms'])" $O/prio_$pr.json)"
      done ;;
    envbench)
      # one env knob over values (ENV_NAME, ENV_VALS), the pipelined bench of ${CFG:-c2} per value
      for v in ${ENV_VALS}; do
        export ${ENV_NAME}=$v
        run timeout -k 10 300 python3 bench.py --config ${CFG:-c2} --no-cpu-baseline > $O/eb_$v.json 2> $O/eb_$v.err \
          || { tail -30 $O/eb_$v.err; exit 1; }
        unset ${ENV_NAME}
        echo "${ENV_NAME}=$v: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['probe_ms'], d['probe_ms_in_step'], d['build_ms'])" $O/eb_$v.json)"
      done ;;
    pcie)
      run timeout -k 10 400 python3 tools/pcie_rate.py > $O/pcie.json 2> $O/pcie.err || { tail -30 $O/pcie.err; exit 1; }
      cat $O/pcie.json ;;
    distprof)
      run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/dist -o d --output-format csv \
        -- python3 bench.py --force-dist --no-cpu-baseline --steps 5 > $O/distprof.json 2> $O/distprof.err \
        || { tail -30 $O/distprof.err; exit 1; } ;;
    kp)
      # per-kernel times of one build + 5 probes (tools/probe_one.py $KP_ARGS), serialized
      run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kp${KP_TAG} -o kp --output-format csv \
        -- python3 tools/probe_one.py ${KP_ARGS} > $O/kp${KP_TAG}.log 2>&1 || { tail -30 $O/kp${KP_TAG}.log; exit 1; }
      tail -1 $O/kp${KP_TAG}.log
      python3 tools/kstats.py $O/kp${KP_TAG} ;;
    abl)
      # ablations of one config's probe ($ABL_ARGS for probe_one.py): DFP_HJ_SL_DBG values
      for d in ${ABL_DBG:-0 1 8}; do
        DFP_HJ_SL_DBG=$d run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/abl$d -o kp --output-format csv \
          -- python3 tools/probe_one.py ${ABL_ARGS} > $O/abl$d.log 2>&1 || { tail -30 $O/abl$d.log; exit 1; }
        echo "DFP_HJ_SL_DBG=$d"; python3 tools/kstats.py $O/abl$d | grep -E "sl_|hs_"
      done ;;
    sqpmc)
      # SQ counters of one build + 5 probes (tools/probe_one.py $KP_ARGS): where the waves wait
      run timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU -d $O/sq${KP_TAG} -o sq --output-format csv \
        -- python3 tools/probe_one.py ${KP_ARGS} > $O/sq${KP_TAG}.log 2>&1 || { tail -30 $O/sq${KP_TAG}.log; exit 1; }
      python3 tools/sq_summary.py $O/sq${KP_TAG} ;;
    envsweep)
      # one env knob over values (ENV_NAME, ENV_VALS): kernel stats of tools/probe_one.py ${KP_ARGS}
      for v in ${ENV_VALS}; do
        export ${ENV_NAME}=$v
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ev_$v -o kp --output-format csv \
          -- python3 tools/probe_one.py ${KP_ARGS} > $O/ev_$v.log 2>&1 || { tail -30 $O/ev_$v.log; exit 1; }
        unset ${ENV_NAME}
        echo "${ENV_NAME}=$v"; python3 tools/kstats.py $O/ev_$v | grep -E "${ENV_GREP:-.}"
      done ;;
    chunk)
      # the sliced probe in K chunks (tools/chunk_probe.py), auto strategy and forced sliced
      run timeout -k 10 200 python3 tools/chunk_probe.py > $O/chunk.log 2>&1 || { tail -30 $O/chunk.log; exit 1; }
      cat $O/chunk.log
      DFP_HJ_PROBE_MODE=sliced run timeout -k 10 200 python3 tools/chunk_probe.py > $O/chunk_sl.log 2>&1 \
        || { tail -30 $O/chunk_sl.log; exit 1; }
      cat $O/chunk_sl.log ;;
    smoke)
      run timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { tail -30 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    trun)
      # the driver's N>1 launch shape, with one rank: stdout must be exactly one JSON line
      run timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 > $O/trun.out 2> $O/trun.err \
        || { tail -30 $O/trun.err; exit 1; }
      wc -l $O/trun.out && python3 -c "import json,sys; json.loads(open(sys.argv[1]).read()); print('one json line ok')" $O/trun.out ;;
    tpch)
      run timeout -k 10 600 python3 tools/bench_tpch.py q3:100 q9:100 > $O/tpch_single.json 2> $O/tpch_single.err \
        || { tail -30 $O/tpch_single.err; exit 1; }
      cat $O/tpch_single.json
      run timeout -k 10 600 python3 tools/bench_tpch.py --dist ${TPCH_DIST:-q3:100 q9:100 q9:300} > $O/tpch_dist.json \
        2> $O/tpch_dist.err || { tail -30 $O/tpch_dist.err; exit 1; }
      cat $O/tpch_dist.json ;;
    dbgshuf)
      run timeout -k 10 300 python3 tools/debug_shuffle.py > $O/dbgshuf.log 2>&1 || { tail -30 $O/dbgshuf.log; exit 1; }
      grep "^n=" $O/dbgshuf.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session $TAG done"
