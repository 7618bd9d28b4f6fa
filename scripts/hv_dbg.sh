#!/bin/bash
# GPU box: reproduce the full-algorithm device run (Walker, seed 0) with the single-tile update kernels and without.
set -o pipefail
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
PGM_DEBUG_TASKS=1 timeout -k 10 300 python scripts/hv_full.py device --env MO-Walker2d-v2 --seeds 0 --ref profiles/r02_hvfull2_oracle_walker.json --out $OUT/hvdbg_one.json > $OUT/hvdbg_one.log 2>&1; echo "ONE rc=$?"; grep -E "debug|Error|Too few" $OUT/hvdbg_one.log | head -20
PGM_NO_ONE=1 PGM_DEBUG_TASKS=1 timeout -k 10 300 python scripts/hv_full.py device --env MO-Walker2d-v2 --seeds 0 --ref profiles/r02_hvfull2_oracle_walker.json --out $OUT/hvdbg_noone.json > $OUT/hvdbg_noone.log 2>&1; echo "NO_ONE rc=$?"; grep -E "debug|Error|Too few" $OUT/hvdbg_noone.log | head -20
