#!/bin/bash
# GPU box: parity of the 16-row-tile update variants + bench lines per variant.  Usage: bash scripts/t16_check.sh TAG
set -o pipefail
TAG=${1:-t16}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "test_ppo_update and t16" -p no:cacheprovider > $OUT/t16_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/t16_tests_$TAG.log | head -20; tail -30 $OUT/t16_tests_$TAG.log; exit 1; }
tail -1 $OUT/t16_tests_$TAG.log
PGM_UPDATE_SPLIT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_production.py -q -x --timeout 120 --timeout-method thread -k "update" -p no:cacheprovider > $OUT/t16_prod_$TAG.log 2>&1 || { echo PROD FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/t16_prod_$TAG.log | head -20; tail -30 $OUT/t16_prod_$TAG.log; exit 1; }
tail -1 $OUT/t16_prod_$TAG.log
for V in 2 3 4; do for P in 40 20 5; do
  PGM_UPDATE_SPLIT=$V timeout -k 10 200 python -u bench.py --scaling strong --tasks $P --steps 6 --warmup 2 --no-cpu-baseline > $OUT/bench_${TAG}_v${V}_p$P.json 2> $OUT/bench_${TAG}_v${V}_p$P.err || { echo BENCH $V $P FAILED; tail -5 $OUT/bench_${TAG}_v${V}_p$P.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${TAG}_v${V}_p$P.json'));print('split $V P=$P', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],2),'ms/step upd', round(d['roofline']['avg_launch_ms'],3), 'frac', round(d['roofline']['frac'],3))"
done; done
