#!/bin/bash
# r05j: compact feature-split fragments (6 blocks per wave at obs_dim <= 20): full GPU suite, A/B against the previous
# fs unit (libpgm_prev), device side of the 40-seed Walker and the 5-seed Humanoid equal-budget HV comparisons
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/r05j_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR)" $OUT/r05j_gpu_tests.log | head -20; tail -30 $OUT/r05j_gpu_tests.log; exit 1; }
tail -1 $OUT/r05j_gpu_tests.log
bash scripts/ab.sh r05j "libpgm libpgm_prev" 3 "" "--env-name MO-HalfCheetah-v2 --tasks 20" "--tasks 5" > /dev/null || exit 1
cat $OUT/ab_r05j.txt
timeout -k 10 900 python -u scripts/hv_full.py device --env MO-Walker2d-v2 --seeds $(seq 0 39) --ref profiles/r05_hvfull_oracle_walker.json --out $OUT/r05_hvfull_walker.json > $OUT/r05j_hv_walker.log 2>&1 || { echo HV WALKER FAILED; tail -20 $OUT/r05j_hv_walker.log; exit 1; }
tail -3 $OUT/r05j_hv_walker.log
timeout -k 10 900 python -u scripts/hv_full.py device --env MO-Humanoid-v2 --seeds 0 1 2 3 4 --ref profiles/r05_hvfull_oracle_humanoid.json --out $OUT/r05_hvfull_humanoid.json > $OUT/r05j_hv_humanoid.log 2>&1 || { echo HV HUMANOID FAILED; tail -20 $OUT/r05j_hv_humanoid.log; exit 1; }
tail -3 $OUT/r05j_hv_humanoid.log
echo all done
