#!/bin/bash
# PMC traffic passes of the C2 bench (FETCH_SIZE and WRITE_SIZE in separate runs) at HEAD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc2; mkdir -p $O
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr -d $O/pmc_c2/pmc_$ctr -o pmc --output-format csv -- python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_c2_$ctr.log 2>&1 || { echo "FAILED $ctr"; exit 1; }
done
echo pmc done
