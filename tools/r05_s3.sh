#!/bin/bash
# r05: kernel + copy trace of the one-rank native radix plan
set -o pipefail
OUT=gpurun_out/${1:-r05f}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 1 2; do
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/kt_radix_c$c -o kt -- \
      python3 bench.py --force-dist --plan radix --comms $c --no-cpu-baseline --steps 10 --warmup 5 > $OUT/kt_radix_c$c.log 2>&1 || exit $?
done
