#!/bin/bash
# r05f: the round-5 HEAD (actor loss two tiles per pass): A/B against the previous HEAD (libpgm_prev), the -m gpu
# suite, smoke, the default bench line, kernel stats, every BASELINE config, PMC of four fs launches, phase stamps,
# and the device side of the long-budget Walker HV comparison (8 seeds, 12 + 2x12 iterations)
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
rm -f $OUT/ab_r05f.txt
bash scripts/ab.sh r05f "libpgm libpgm_prev" 2 "" "--env-name MO-HalfCheetah-v2 --tasks 20" > /dev/null || exit 1
cat $OUT/ab_r05f.txt
bash scripts/round_check.sh r05f || exit 1
bash scripts/configs_check.sh r05f || exit 1
bash scripts/pmc.sh r05f_walker_p40 > /dev/null && \
bash scripts/pmc.sh r05f_cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 > /dev/null && \
bash scripts/pmc.sh r05f_hopper3_p27 --env-name MO-Hopper-v3 --tasks 27 > /dev/null && \
bash scripts/pmc.sh r05f_walker_p5 --tasks 5 > /dev/null || { echo PMC FAILED; exit 1; }
for f in gpurun_out/pmc_r05f_*.json; do python -c "import json;d=json.load(open('$f'));print('$f', d['variant'], d['source_hash'], round(d['hbm_bytes_per_launch']/1e9,3),'GB')"; done
for cfg in "MO-Walker2d-v2 5" "MO-Walker2d-v2 40" "MO-HalfCheetah-v2 20"; do
  set -- $cfg
  ENV=$1 P=$2 STAMP_BLOCK=8 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > gpurun_out/r05f_stamps_$1_$2.txt 2>&1 || { echo STAMPS FAILED; tail gpurun_out/r05f_stamps_$1_$2.txt; exit 1; }
done
timeout -k 10 900 python -u scripts/hv_full.py device --env MO-Walker2d-v2-long --seeds 0 1 2 3 4 5 6 7 --ref profiles/r05_hvfull_oracle_walkerlong.json --out $OUT/r05_hvfull_walkerlong.json > $OUT/r05f_hv_walkerlong.log 2>&1 || { echo HV LONG FAILED; tail -20 $OUT/r05f_hv_walkerlong.log; exit 1; }
tail -c 600 $OUT/r05f_hv_walkerlong.log
echo all done
