#!/bin/bash
# r05p: dW1 inputs 16.. on the VALU (compact fs) + back-to-back first polls: fs / exchange / production GPU tests,
# A/B libpgm (both) vs libpgm_tail (VALU tail only) vs libpgm_prev (HEAD)
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fs.py tests/test_gpu_exchange.py tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r05p_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/r05p_gpu_tests.log; exit 1; }
tail -1 $OUT/r05p_gpu_tests.log
rm -f $OUT/ab_r05p.txt
bash scripts/ab.sh r05p "libpgm libpgm_tail libpgm_prev" 2 "" "--env-name MO-HalfCheetah-v2 --tasks 20" "--tasks 5" > /dev/null || exit 1
cat $OUT/ab_r05p.txt
