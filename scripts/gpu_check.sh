#!/bin/bash
# GPU box routine: build, parity tests, smoke, bench, rocprof kernel stats.  Usage: scripts/gpu_check.sh TAG [bench args]
set -o pipefail
TAG=${1:-run}; shift
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
python -m pgmorl_amd.build > $OUT/build.log 2>&1 || { echo BUILD FAILED; tail -20 $OUT/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1
TRC=$?
tail -3 $OUT/gpu_tests_$TAG.log
[ $TRC -eq 0 ] || { echo TESTS FAILED rc=$TRC; grep -E "^(FAILED|ERROR)|Error|assert" $OUT/gpu_tests_$TAG.log | head -30; }
[ $TRC -le 1 ] || exit $TRC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke_$TAG.log; exit 1; }
timeout -k 10 400 python bench.py "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo BENCH FAILED; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o $TAG --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_$TAG.log; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$OUT/prof_$TAG/**/*kernel_stats.csv',recursive=True)[0]
for x in csv.DictReader(open(f)):
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1),'us', x['Percentage'])
PY
