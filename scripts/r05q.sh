#!/bin/bash
# r05q: layer-1 inputs 16.. on the VALU too (compact fs): fs / exchange / production GPU tests,
# A/B libpgm (VALU tails in layer 1 and dW1) vs libpgm_tail (dW1 tail only)
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fs.py tests/test_gpu_exchange.py tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r05q_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/r05q_gpu_tests.log; exit 1; }
tail -1 $OUT/r05q_gpu_tests.log
rm -f $OUT/ab_r05q.txt
bash scripts/ab.sh r05q "libpgm libpgm_tail" 3 "" "--env-name MO-HalfCheetah-v2 --tasks 20" "--tasks 5" > /dev/null || exit 1
cat $OUT/ab_r05q.txt
