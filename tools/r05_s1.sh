#!/bin/bash
# r05 session 1: the multi-GPU C plans at W = 1/2/4/8 (thread transport) + one-rank RCCL lines
set -o pipefail
OUT=gpurun_out/${1:-r05a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v --maxfail=5 --timeout 240 --timeout-method thread \
    tests/test_gpu_dist_threads.py tests/test_gpu_sharded_build.py tests/test_gpu_distributed.py > $OUT/tests.log 2>&1 || exit $?
for plan in sharded radix; do
  for nat in auto off; do
    timeout -k 10 300 python bench.py --force-dist --plan $plan --native $nat --no-cpu-baseline --steps 20 --warmup 10 \
        > $OUT/bench_${plan}_${nat}.json 2> $OUT/bench_${plan}_${nat}.err || exit $?
  done
done
