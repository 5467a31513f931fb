#!/bin/bash
# r05: native radix / sharded one-rank lines after the job-free fix
set -o pipefail
OUT=gpurun_out/${1:-r05o}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_gpu_dist_threads.py tests/test_gpu_sharded_build.py tests/test_gpu_distributed.py > $OUT/tests.log 2>&1 || exit $?
tail -1 $OUT/tests.log
B="python bench.py --force-dist --no-cpu-baseline --steps 20 --warmup 10"
run() { name=$1; shift; timeout -k 10 300 env "$@" > $OUT/$name.json 2> $OUT/$name.err || exit $?;
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k:d.get(k) for k in ['value','ms_per_step','probe_ms','build_ms','exchange_ms','host_ms_per_step']})" $OUT/$name.json $name; }
run radix_c1 DFP_X=0 $B --plan radix --comms 1
run radix_c2 DFP_X=0 $B --plan radix --comms 2
run radix_machinery DFP_HJ_DIST_W1_IDENTITY=0 $B --plan radix --comms 1
run radix_off DFP_X=0 $B --plan radix --native off
run sharded_c2 DFP_X=0 $B --plan sharded
run sharded_machinery DFP_HJ_DIST_W1_IDENTITY=0 $B --plan sharded
