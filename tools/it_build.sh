set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/it4; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@" || { echo "FAILED($?): $*"; exit 1; }; }
step 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
for c in c2 c3 c2h; do
  step 300 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
  DFP_HJ_MODFRAG=0 step 300 python3 bench.py --config $c --no-cpu-baseline > $O/bench_${c}_old.json 2> $O/bench_${c}_old.err
  for f in $O/bench_$c.json $O/bench_${c}_old.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['probe_ms'], d.get('build_ms'), d['roofline']['frac'])" $f; done
done
step 300 rocprofv3 --kernel-trace --stats -d $O/ks_c2 -o ks --output-format csv -- python3 bench.py --config c2 --no-cpu-baseline --same-stream --sync-steps --steps 5 --warmup 3 > $O/ks_c2.json 2> $O/ks_c2.err
python3 tools/kstats.py $O/ks_c2 > $O/ks_c2.txt; head -14 $O/ks_c2.txt
