#!/bin/bash
# r05g: round-5 final state: the -m gpu suite, smoke, default bench line, kernel stats, every BASELINE config, PMC of
# four fs launches at the final source hash, and the device side of the 10-seed Humanoid HV comparison
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
bash scripts/round_check.sh r05g || exit 1
bash scripts/configs_check.sh r05g || exit 1
bash scripts/pmc.sh r05g_walker_p40 > /dev/null && \
bash scripts/pmc.sh r05g_cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 > /dev/null && \
bash scripts/pmc.sh r05g_hopper3_p27 --env-name MO-Hopper-v3 --tasks 27 > /dev/null && \
bash scripts/pmc.sh r05g_walker_p5 --tasks 5 > /dev/null || { echo PMC FAILED; exit 1; }
for f in gpurun_out/pmc_r05g_*.json; do python -c "import json;d=json.load(open('$f'));print('$f', d['variant'], d['source_hash'], round(d['hbm_bytes_per_launch']/1e9,3),'GB')"; done
timeout -k 10 900 python -u scripts/hv_full.py device --env MO-Humanoid-v2 --seeds 0 1 2 3 4 5 6 7 8 9 --ref profiles/r05_hvfull_oracle_humanoid.json --out $OUT/r05_hvfull_humanoid.json > $OUT/r05g_hv_humanoid.log 2>&1 || { echo HV HUMANOID FAILED; tail -20 $OUT/r05g_hv_humanoid.log; exit 1; }
tail -c 300 $OUT/r05g_hv_humanoid.log
echo all done
