#!/bin/bash
# r05o: SQ counters (MFMA busy share, instruction mix, LDS bank conflicts, wait shares) of the compact fs update at
# Walker P = 40 (NS 6, R 3, two per CU), HalfCheetah P = 20 (NS 8, R 2, two per CU), Walker P = 5 (NS 16, R 1)
set -o pipefail
bash scripts/sq_counters.sh r05o_fs_walker_p40 > /dev/null && \
bash scripts/sq_counters.sh r05o_fs_cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 > /dev/null && \
bash scripts/sq_counters.sh r05o_fs_walker_p5 --tasks 5 > /dev/null || exit 1
for f in gpurun_out/sq_r05o_*.json; do echo "== $f"; cat $f; echo; done
