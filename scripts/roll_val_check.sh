#!/bin/bash
# GPU box: rollout / value / iteration / production parity, then the headline bench with rocprof kernel stats.
set -o pipefail
TAG=${1:-rv}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py tests/test_gpu_production.py -k "rollout or value or iteration or golden or production" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/rv_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/rv_tests_$TAG.log | head -20; tail -20 $OUT/rv_tests_$TAG.log; exit 1; }
tail -1 $OUT/rv_tests_$TAG.log
bash scripts/bench_prof.sh $TAG > $OUT/bp_$TAG.txt 2>&1 || { echo PROF FAILED; tail $OUT/bp_$TAG.txt; exit 1; }
head -c 300 $OUT/bp_$TAG.txt; echo; grep -E "gae|update|rollout|value|adv" $OUT/bp_$TAG.txt
