#!/bin/bash
# GPU box: the -m gpu suite on the default libpgm.so, then bench lines of the default and A/B variant libraries.
# Usage: bash scripts/ab_check.sh TAG "lib:tasks" ...   (e.g. libpgm:40 libpgm_var40:40)
set -o pipefail
TAG=$1; shift
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/gpu_tests_$TAG.log | head -20; tail -30 $OUT/gpu_tests_$TAG.log; exit 1; }
tail -1 $OUT/gpu_tests_$TAG.log
bash scripts/var_bench.sh $TAG "$@"
