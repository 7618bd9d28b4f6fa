#!/bin/bash
# r05h: every BASELINE config's per-GPU load + strong-scaling loads, rocprofv3 kernel stats of the headline, PMC
# (FETCH_SIZE / WRITE_SIZE, separate passes) of the update kernel at Walker P = 40, HalfCheetah P = 20, Hopper-v3 P = 27,
# Walker P = 5
set -o pipefail
bash scripts/configs_check.sh r05h || exit 1
bash scripts/bench_prof.sh r05h > gpurun_out/bp_r05h.txt 2>&1 || { echo PROF FAILED; tail gpurun_out/bp_r05h.txt; exit 1; }
tail -8 gpurun_out/bp_r05h.txt
bash scripts/pmc.sh r05h_walker_p40 > /dev/null && \
bash scripts/pmc.sh r05h_cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 > /dev/null && \
bash scripts/pmc.sh r05h_hopper3_p27 --env-name MO-Hopper-v3 --tasks 27 > /dev/null && \
bash scripts/pmc.sh r05h_walker_p5 --tasks 5 > /dev/null || { echo PMC FAILED; exit 1; }
for f in gpurun_out/pmc_r05h_*.json; do python -c "import json;d=json.load(open('$f'));print('$f', d['variant'], round(d['hbm_bytes_per_launch']/1e9,3),'GB')"; done
