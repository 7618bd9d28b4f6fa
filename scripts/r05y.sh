#!/bin/bash
# r05y: actor loss two tiles per pass (8-lane row sums):
# fs / exchange / production GPU tests, A/B against HEAD (libpgm_prev), actor vs critic stamps
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fs.py tests/test_gpu_exchange.py tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r05y_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/r05y_gpu_tests.log; exit 1; }
tail -1 $OUT/r05y_gpu_tests.log
rm -f $OUT/ab_r05y.txt
bash scripts/ab.sh r05y "libpgm libpgm_prev" 3 "" "--env-name MO-HalfCheetah-v2 --tasks 20" "--tasks 5" > /dev/null || exit 1
cat $OUT/ab_r05y.txt
bash scripts/r05s.sh
