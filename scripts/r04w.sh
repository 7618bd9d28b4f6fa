#!/bin/bash
# GPU box: the split rollout (chain and objective workgroups): rollout parity, production, whole-run tests, then the
# rollout timing split vs one workgroup (PGM_ROLL_SPLIT=0).
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_production.py tests/test_gpu_morl.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r04w_tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/r04w_tests.log | head; tail -30 $OUT/r04w_tests.log; exit 1; }
tail -2 $OUT/r04w_tests.log
timeout -k 10 300 python -u scripts/roll_time.py pgmorl_amd/libpgm.so pgmorl_amd/libpgm.so 2>&1 | grep rollout_ms
PGM_ROLL_SPLIT=0 timeout -k 10 300 python -u scripts/roll_time.py pgmorl_amd/libpgm.so 2>&1 | grep rollout_ms
