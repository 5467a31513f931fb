#!/bin/bash
# Round 4: forced one-rank multi-GPU bench lines (build_ms from events on the build stream,
# probe_ms on the probe stream, host_ms_per_step), the sharded plan with its build side
# through the C ABI (RCCL in hj_dist.cpp) and through torch.distributed, and the TPC-H
# Q9 SF300 lines: one GPU, 8 radix shards on the GPU, and a device budget that shards the
# large builds. Every GPU step under its own timeout; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04m}; mkdir -p $O
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
for pl in sharded radix broadcast; do
  step 240 python3 bench.py --force-dist --plan $pl --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_$pl.json 2> $O/bench_$pl.err
  cat $O/bench_$pl.json
done
step 240 python3 bench.py --force-dist --plan sharded --native off --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_sharded_py.json 2> $O/bench_sharded_py.err
cat $O/bench_sharded_py.json
step 300 python3 tools/bench_tpch.py --reps 3 q9:300 > $O/tpch_single.json 2> $O/tpch_single.err
cat $O/tpch_single.json
step 300 python3 tools/bench_tpch.py --reps 3 --shards 8 q9:300 > $O/tpch_shards.json 2> $O/tpch_shards.err
cat $O/tpch_shards.json
step 300 python3 tools/bench_tpch.py --reps 3 --budget 8000000000 q9:300 > $O/tpch_budget.json 2> $O/tpch_budget.err
cat $O/tpch_budget.json
