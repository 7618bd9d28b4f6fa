#!/bin/bash
# GPU box: A/B of the update kernels per per-GPU load (default launcher choice vs PGM_UPDATE_KERNEL=fs).
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
for P in 5 10 20 40; do
  run p${P}_def '' --scaling strong --tasks $P && run p${P}_fs PGM_UPDATE_KERNEL=fs --scaling strong --tasks $P || exit 1
done
run cheetah20_def '' --env-name MO-HalfCheetah-v2 --tasks 20 && run cheetah20_fs PGM_UPDATE_KERNEL=fs --env-name MO-HalfCheetah-v2 --tasks 20 && \
run hopper2_p5_def '' --env-name MO-Hopper-v2 --tasks 5 --num-processes 1 && run hopper2_p5_fs PGM_UPDATE_KERNEL=fs --env-name MO-Hopper-v2 --tasks 5 --num-processes 1
