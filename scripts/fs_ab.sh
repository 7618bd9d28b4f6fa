#!/bin/bash
# GPU box: A/B of the update kernels per per-GPU load: the launcher's default (auto: the feature-split update where it
# gets >= 4 parts per tower) vs the row-split kernels (PGM_UPDATE_KERNEL=mfma), the tagged parameter hop
# (PGM_FS_PTAG=1), fewer parts at P = 5 (PGM_FS_NS=8) and the feature-split update forced at P = 40.
# Usage: bash scripts/fs_ab.sh TAG
set -o pipefail
TAG=${1:-ab}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
run() {  # name, env assignment ('' = default), bench args...
  local n=$1 e=$2; shift 2
  env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-whole-run --no-strong "$@" > $OUT/ab_${TAG}_$n.json 2> $OUT/ab_${TAG}_$n.err || { echo BENCH $n FAILED; tail -5 $OUT/ab_${TAG}_$n.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/ab_${TAG}_$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],3),'ms/step', r['kernel'], round(r['avg_launch_ms'],3),'ms frac', round(r['frac'],3))"
}
# the tagged parameter hop first: a timed-out exchange is a handled error (the word names the wait), not a GPU fault
run p5_ptag PGM_FS_PTAG=1 --scaling strong --tasks 5 || echo "p5_ptag failed (handled), continuing"
for P in 5 10 20; do run p${P}_def '' --scaling strong --tasks $P || exit 1; done
run p5_ns8 "PGM_UPDATE_KERNEL=fs PGM_FS_NS=8" --scaling strong --tasks 5 && \
run p40_def '' --scaling strong --tasks 40 && run p40_fs PGM_UPDATE_KERNEL=fs --scaling strong --tasks 40 && \
run hopper2_p5_def '' --env-name MO-Hopper-v2 --tasks 5 --num-processes 1 || exit 1
