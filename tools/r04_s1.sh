#!/bin/bash
# Round 4, first GPU session: the new tests first (device budget, SF300 Q9 on 8 shards,
# operator over a multi-GPU table), then the whole GPU suite, the forced one-rank multi-GPU
# bench lines (build_ms / host_ms_per_step now measured), the C2 bench line and the SF300
# Q9 TPC-H lines (one GPU, 8 radix shards, device budget). Every GPU step under its own
# timeout; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s1; mkdir -p $O
step() { local t=$1; shift; echo "== $*"; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
PT="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
step 600 $PT tests/test_gpu_sharded_build.py tests/test_gpu_operator.py tests/test_gpu_tpch.py -k "budget or multi_gpu or sf300 or one_rank or native" > $O/new_tests.log 2>&1
tail -2 $O/new_tests.log
step 900 $PT tests -m gpu > $O/tests.log 2>&1
tail -2 $O/tests.log
for pl in sharded radix broadcast; do
  step 300 python3 bench.py --force-dist --plan $pl --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_$pl.json 2> $O/bench_$pl.err
  cat $O/bench_$pl.json
done
step 300 python3 bench.py --force-dist --plan sharded --native off --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_sharded_py.json 2> $O/bench_sharded_py.err
cat $O/bench_sharded_py.json
step 300 python3 bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
cat $O/bench_c2.json
step 600 python3 tools/bench_tpch.py --reps 3 q9:300 > $O/tpch_single.json 2> $O/tpch_single.err
step 600 python3 tools/bench_tpch.py --reps 3 --shards 8 q9:300 > $O/tpch_shards.json 2> $O/tpch_shards.err
step 600 python3 tools/bench_tpch.py --reps 3 --budget 8000000000 q9:300 > $O/tpch_budget.json 2> $O/tpch_budget.err
cat $O/tpch_*.json
