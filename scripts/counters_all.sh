#!/bin/bash
# GPU box: SQ counter passes (scripts/sq_counters.sh) of the three update kernels at their headline loads -- MODE 2
# (Walker P=40), t16 (HalfCheetah P=20), wide (Humanoid P=20, N=8) -- and FETCH/WRITE_SIZE of the t16 and wide
# launches (scripts/pmc.sh).  Usage: bash scripts/counters_all.sh TAG
set -o pipefail
TAG=${1:-c}
bash scripts/sq_counters.sh ${TAG}_mode2_walker_p40 > /dev/null && \
bash scripts/sq_counters.sh ${TAG}_t16_cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 > /dev/null && \
bash scripts/sq_counters.sh ${TAG}_wide_humanoid_p20 --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 > /dev/null && \
bash scripts/pmc.sh ${TAG}_cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 > /dev/null && \
bash scripts/pmc.sh ${TAG}_walker_p40 > /dev/null && \
python - <<PY
import json, glob
for f in sorted(glob.glob('gpurun_out/sq_${TAG}_*.json')) + sorted(glob.glob('gpurun_out/pmc_${TAG}_*.json')):
    d = json.load(open(f))
    keys = ('kernel_ns_profiled', 'mfma_busy_share', 'per_wave', 'clock_ghz', 'lds_bank_conflict_per_active_lds',
            'total_bytes', 'bytes_per_launch', 'hbm_bytes_per_launch')
    print(f, {k: d[k] for k in keys if k in d})
PY
