#!/bin/bash
# r05r: compact fs fragments + VALU input tails at HEAD: the -m gpu suite, smoke, the default bench line (cpu baseline + whole run),
# rocprofv3 kernel stats, every BASELINE config's per-GPU load, PMC (FETCH_SIZE / WRITE_SIZE, separate passes) of the
# update at Walker P = 40 / 5, HalfCheetah P = 20, Hopper-v3 P = 27
set -o pipefail
bash scripts/round_check.sh r05r || exit 1
bash scripts/configs_check.sh r05r || exit 1
bash scripts/pmc.sh r05r_walker_p40 > /dev/null && \
bash scripts/pmc.sh r05r_cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 > /dev/null && \
bash scripts/pmc.sh r05r_hopper3_p27 --env-name MO-Hopper-v3 --tasks 27 > /dev/null && \
bash scripts/pmc.sh r05r_walker_p5 --tasks 5 > /dev/null || { echo PMC FAILED; exit 1; }
for f in gpurun_out/pmc_r05r_*.json; do python -c "import json;d=json.load(open('$f'));print('$f', d['variant'], d['source_hash'], round(d['hbm_bytes_per_launch']/1e9,3),'GB')"; done
for cfg in "MO-Walker2d-v2 5" "MO-Walker2d-v2 40" "MO-HalfCheetah-v2 20"; do
  set -- $cfg
  ENV=$1 P=$2 STAMP_BLOCK=0 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > gpurun_out/r05r_stamps_$1_$2.txt 2>&1 || { echo STAMPS FAILED; tail gpurun_out/r05r_stamps_$1_$2.txt; exit 1; }
  echo "=== $1 P=$2"; grep -A17 "== fs" gpurun_out/r05r_stamps_$1_$2.txt
done
