#!/bin/bash
# GPU box: rollout parity (lane kernel), phase stamps of the rollout, quick bench line.  Usage: bash scripts/roll_check.sh TAG
set -o pipefail
TAG=${1:-roll}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py tests/test_gpu_production.py -q -x --timeout 120 --timeout-method thread -k "rollout or mopg or golden or iteration or overlapped" -p no:cacheprovider > $OUT/roll_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/roll_tests_$TAG.log | head -20; tail -30 $OUT/roll_tests_$TAG.log; exit 1; }
tail -1 $OUT/roll_tests_$TAG.log
PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/stamps_$TAG.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/stamps_$TAG.txt; exit 1; }
grep -A12 "== lanes" $OUT/stamps_$TAG.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo BENCH FAILED; tail -20 $OUT/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print('bench', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],2),'ms/step upd', round(d['roofline']['avg_launch_ms'],2))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o $TAG --output-format csv -- python $OLDPWD/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_$TAG.log; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$OUT/prof_$TAG/**/*kernel_stats.csv',recursive=True)[0]
for x in csv.DictReader(open(f)):
    if float(x['Percentage']) > 0.05:
        print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1),'us', x['Percentage'])
PY
