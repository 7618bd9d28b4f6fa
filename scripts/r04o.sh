#!/bin/bash
# GPU box: round check (GPU suite, smoke, bench + rocprof), per-config bench lines, PMC of the feature-split update
# at HalfCheetah P = 20 and Walker P = 5.
set -o pipefail
bash scripts/round_check.sh r04o || exit 1
bash scripts/configs_check.sh r04o || exit 1
bash scripts/pmc.sh r04o_cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 || exit 1
bash scripts/pmc.sh r04o_walker_p5 --scaling strong --tasks 5 || exit 1
