#!/bin/bash
# r05 session 2: one-rank lines of the native plans
set -o pipefail
OUT=gpurun_out/${1:-r05c}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_gpu_dist_threads.py \
    tests/test_gpu_sharded_build.py tests/test_gpu_distributed.py > $OUT/tests.log 2>&1 || exit $?
B="python bench.py --force-dist --no-cpu-baseline --steps 20 --warmup 10"
run() { name=$1; shift; timeout -k 10 300 env "$@" > $OUT/$name.json 2> $OUT/$name.err || exit $?; }
run sharded_c1 DFP_X=0 $B --plan sharded --comms 1
run sharded_c2 DFP_X=0 $B --plan sharded --comms 2
run sharded_off DFP_X=0 $B --plan sharded --native off
run radix_c1 DFP_X=0 $B --plan radix --comms 1
run radix_c2 DFP_X=0 $B --plan radix --comms 2
run radix_off DFP_X=0 $B --plan radix --native off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/kt_sharded -o kt -- \
      python3 bench.py --force-dist --plan sharded --no-cpu-baseline --steps 10 --warmup 5 > $OUT/kt_sharded.log 2>&1 || exit $?
