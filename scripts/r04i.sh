#!/bin/bash
# GPU box: rollout parity (kernels, production, whole MORL run) after moving the action side to the objective waves,
# then rollout timing A/B: HEAD vs PGM_EXP 48 (everything on the chain) vs 44 (layer-2 inputs by an LDS row).
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_production.py tests/test_gpu_morl.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r04i_tests.log 2>&1 || { tail -30 $OUT/r04i_tests.log; exit 1; }
tail -2 $OUT/r04i_tests.log
timeout -k 10 300 python -u scripts/roll_time.py pgmorl_amd/libpgm.so pgmorl_amd/libpgm_var48.so pgmorl_amd/libpgm_var44.so > $OUT/r04i_roll.txt 2>&1 || { tail $OUT/r04i_roll.txt; exit 1; }
cat $OUT/r04i_roll.txt
