#!/bin/bash
# GPU box: GAE / advantage / iteration parity, then the headline bench with rocprof kernel stats.
set -o pipefail
TAG=${1:-gae}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py tests/test_gpu_morl.py -k "gae or adv or golden or iteration or mopg or morl" -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gae_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/gae_tests_$TAG.log | head -20; tail -20 $OUT/gae_tests_$TAG.log; exit 1; }
tail -1 $OUT/gae_tests_$TAG.log
bash scripts/bench_prof.sh $TAG > $OUT/bp_$TAG.txt 2>&1 || { echo PROF FAILED; tail $OUT/bp_$TAG.txt; exit 1; }
head -c 400 $OUT/bp_$TAG.txt; echo; grep -E "gae|update|rollout|value|adv" $OUT/bp_$TAG.txt
