#!/bin/bash
# r05: one-rank sharded line after the one-rank identity path
set -o pipefail
OUT=gpurun_out/${1:-r05g}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_gpu_sharded_build.py tests/test_gpu_dist_threads.py > $OUT/tests.log 2>&1 || exit $?
B="python bench.py --force-dist --no-cpu-baseline --steps 20 --warmup 10"
run() { name=$1; shift; timeout -k 10 300 env "$@" > $OUT/$name.json 2> $OUT/$name.err || exit $?; }
run sharded DFP_X=0 $B --plan sharded
run sharded_machinery DFP_HJ_DIST_W1_IDENTITY=0 $B --plan sharded
run sharded_off DFP_X=0 $B --plan sharded --native off
