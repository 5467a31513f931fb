#!/bin/bash
# Round-3 closing measurement set on one MI355X (run from the repo root via gpurun): the GPU
# test suite and smoke, bench lines (C2 with the CPU baseline, C2h, C3, the forced one-rank
# multi-GPU plans), serialized and pipelined kernel traces, PMC traffic passes (FETCH_SIZE
# and WRITE_SIZE in separate runs). Every GPU step under its own timeout; stops at the first
# failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final2; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
step 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
step 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
step 400 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err
step 400 python3 bench.py --config c2h --no-cpu-baseline > $O/bench_c2h.json 2> $O/bench_c2h.err
step 400 python3 bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err
for pl in radix broadcast sharded; do
  step 300 python3 bench.py --force-dist --plan $pl --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_$pl.json 2> $O/bench_$pl.err
done
echo bench done
for c in c2 c2h c3; do
  step 300 rocprofv3 --kernel-trace --stats -d $O/kt_$c -o kt --output-format csv -- python3 bench.py --config $c --no-cpu-baseline > $O/kt_$c.json 2> $O/kt_$c.err
  step 300 rocprofv3 --kernel-trace --stats -d $O/ks_$c -o ks --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --same-stream --sync-steps --steps 5 --warmup 3 > $O/ks_$c.json 2> $O/ks_$c.err
done
echo traces done
for c in c2 c2h c3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    step 300 rocprofv3 --pmc $ctr -d $O/pmc_$c/pmc_$ctr -o pmc --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_${c}_$ctr.log 2>&1
  done
done
echo pmc done
