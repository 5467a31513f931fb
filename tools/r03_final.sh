#!/bin/bash
# Round-3 measurement set on one MI355X (run from the repo root via gpurun): bench lines,
# kernel traces and PMC traffic passes. Every GPU step under its own timeout; stops at the
# first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
step 400 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err
step 400 python3 bench.py --config c2h > $O/bench_c2h.json 2> $O/bench_c2h.err
step 400 python3 bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err
step 300 python3 bench.py --force-dist --plan radix --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_radix.json 2> $O/bench_radix.err
step 300 python3 bench.py --force-dist --plan broadcast --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_bcast.json 2> $O/bench_bcast.err
echo bench done
for c in c2 c2h c3; do
  step 300 rocprofv3 --kernel-trace --stats -d $O/kt_$c -o kt --output-format csv -- python3 bench.py --config $c --no-cpu-baseline > $O/kt_$c.json 2> $O/kt_$c.err
  step 300 rocprofv3 --kernel-trace --stats -d $O/ks_$c -o ks --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --same-stream --sync-steps --steps 5 --warmup 3 > $O/ks_$c.json 2> $O/ks_$c.err
done
step 300 rocprofv3 --kernel-trace --stats -d $O/kt_radix -o kt --output-format csv -- python3 bench.py --force-dist --plan radix --no-cpu-baseline --steps 10 --warmup 5 > $O/kt_radix.json 2> $O/kt_radix.err
echo traces done
for c in c2 c2h c3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    step 300 rocprofv3 --pmc $ctr -d $O/pmc_$c/pmc_$ctr -o pmc --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_${c}_$ctr.log 2>&1
  done
done
echo pmc done
