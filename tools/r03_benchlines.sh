#!/bin/bash
# The three single-GPU bench lines (C2 with its CPU baseline, C2h, C3) at HEAD, reading the
# committed traffic profiles; one MI355X via gpurun.
set -o pipefail
O=gpurun_out/lines; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
step 400 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err
step 300 python3 bench.py --config c2h > $O/bench_c2h.json 2> $O/bench_c2h.err
step 300 python3 bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err
cat $O/bench_c2.json
