#!/bin/bash
# GPU box: wide (Humanoid) evaluation kernel parity + Humanoid bench line with kernel stats.
set -o pipefail
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
TAG=${1:-ew}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_production.py -x -q -k "eval" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_evalw_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $OUT/t_evalw_$TAG.log | tail -30; exit 1; }
tail -1 $OUT/t_evalw_$TAG.log
bash scripts/bench_prof.sh hum_$TAG --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 > $OUT/bp_hum_$TAG.txt 2>&1 || { tail -20 $OUT/bp_hum_$TAG.txt; exit 1; }
cat $OUT/bp_hum_$TAG.txt | cut -c1-400
