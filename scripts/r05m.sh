#!/bin/bash
# r05m: two-hop feature-split exchange (replicated Adam, no parameter hand-off): fs / exchange / production GPU tests,
# A/B against the three-hop compact version (libpgm_prev = HEAD pgm_ppo_fs.hip)
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fs.py tests/test_gpu_exchange.py tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r05m_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/r05m_gpu_tests.log; exit 1; }
tail -1 $OUT/r05m_gpu_tests.log
rm -f $OUT/ab_r05m.txt
bash scripts/ab.sh r05m "libpgm libpgm_prev" 2 "" "--env-name MO-HalfCheetah-v2 --tasks 20" "--tasks 5" "--env-name MO-Hopper-v3 --tasks 27" > /dev/null || exit 1
cat $OUT/ab_r05m.txt
