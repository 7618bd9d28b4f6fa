#!/bin/bash
# GPU box: bench line + rocprofv3 kernel stats (no tests).  Usage: scripts/bench_prof.sh TAG [bench args]
set -o pipefail
TAG=${1:-run}; shift
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline --no-whole-run "$@" > $OUT/bench_prof_$TAG.json 2> $OUT/bench_prof_$TAG.err || { echo BENCH FAILED; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
cat $OUT/bench_prof_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o $TAG --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-whole-run "$@" > $OUT/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_$TAG.log; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$OUT/prof_$TAG/**/*kernel_stats.csv',recursive=True)[0]
for x in csv.DictReader(open(f)):
    if float(x['Percentage']) > 0.05:
        print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1),'us', x['Percentage'])
PY
