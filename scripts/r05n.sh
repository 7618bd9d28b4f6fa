#!/bin/bash
# r05n: compact fs fragments at HEAD: the -m gpu suite, smoke, the default bench line (cpu baseline + whole run),
# rocprofv3 kernel stats, every BASELINE config's per-GPU load, PMC (FETCH_SIZE / WRITE_SIZE, separate passes) of the
# update at Walker P = 40 / 5, HalfCheetah P = 20, Hopper-v3 P = 27
set -o pipefail
bash scripts/round_check.sh r05n || exit 1
bash scripts/configs_check.sh r05n || exit 1
bash scripts/pmc.sh r05n_walker_p40 > /dev/null && \
bash scripts/pmc.sh r05n_cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 > /dev/null && \
bash scripts/pmc.sh r05n_hopper3_p27 --env-name MO-Hopper-v3 --tasks 27 > /dev/null && \
bash scripts/pmc.sh r05n_walker_p5 --tasks 5 > /dev/null || { echo PMC FAILED; exit 1; }
for f in gpurun_out/pmc_r05n_*.json; do python -c "import json;d=json.load(open('$f'));print('$f', d['variant'], d['source_hash'], round(d['hbm_bytes_per_launch']/1e9,3),'GB')"; done
