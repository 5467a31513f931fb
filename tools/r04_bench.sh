#!/bin/bash
# Round 4 bench pass: parity tests of the sliced probe, then bench lines of each config in
# CFGS under each environment in VARIANTS ("A=1,B=2" items separated by spaces; "-" = none),
# alternating, twice; serialized kernel stats for the configs in KSTATS.
# OUT names the gpurun_out subdirectory. Every GPU step under its own timeout.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04b}; mkdir -p $O
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
PT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
if [ -z "$NOTEST" ]; then
  step 400 $PT ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_join_types.py} > $O/tests.log 2>&1
  tail -1 $O/tests.log
fi
B="python3 bench.py --no-cpu-baseline"
for cfg in ${CFGS:-c2}; do
  for rep in 1 2; do
    for v in ${VARIANTS:--}; do
      tag=$(echo "$v" | tr ',=' '__')
      envs=$( [ "$v" = "-" ] && echo "" || echo "$v" | tr ',' ' ')
      step 200 env $envs $B --config $cfg > $O/bench_${cfg}_${tag}_$rep.json 2> $O/bench_${cfg}_${tag}_$rep.err
      echo "$cfg [$v] #$rep $(python3 -c "import json; d=json.load(open('$O/bench_${cfg}_${tag}_$rep.json')); print(d['value'], d['ms_per_step'], d.get('probe_ms'), d.get('build_ms'), d['roofline']['frac'])")"
    done
  done
done
for cfg in $KSTATS; do
  step 300 rocprofv3 --kernel-trace --stats -d $O/ks_$cfg -o ks --output-format csv -- python3 bench.py --no-cpu-baseline --config $cfg --same-stream --sync-steps --steps 5 --warmup 3 > $O/ks_$cfg.json 2> $O/ks_$cfg.err
  python3 tools/kstats.py $O/ks_$cfg > $O/ks_$cfg.txt; head -8 $O/ks_$cfg.txt
done
for cfg in $TIMELINE; do
  step 120 python3 tools/timeline_sliced.py --config=$cfg > $O/tl_$cfg.txt 2>&1
  grep -v amdgpu.ids $O/tl_$cfg.txt
done
