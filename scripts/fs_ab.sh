#!/bin/bash
# GPU box: A/B of the update kernels per per-GPU load: the launcher's default (auto: the feature-split update where it
# gets >= 4 parts per tower) vs the row-split kernels (PGM_UPDATE_KERNEL=mfma), then fs phase stamps at P = 5 / 20.
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
  run p${P}_def '' --scaling strong --tasks $P && run p${P}_rows PGM_UPDATE_KERNEL=mfma --scaling strong --tasks $P || exit 1
done
run cheetah20_def '' --env-name MO-HalfCheetah-v2 --tasks 20 && run cheetah20_rows PGM_UPDATE_KERNEL=mfma --env-name MO-HalfCheetah-v2 --tasks 20 && \
run hopper3_27_def '' --env-name MO-Hopper-v3 --tasks 27 && \
run hopper2_p5_def '' --env-name MO-Hopper-v2 --tasks 5 --num-processes 1 && run hopper2_p5_rows PGM_UPDATE_KERNEL=mfma --env-name MO-Hopper-v2 --tasks 5 --num-processes 1 || exit 1
if [ -f pgmorl_amd/libpgm_stamps.so ]; then
for P in 5 20; do
  P=$P STAMP_BLOCK=1 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/stamps_${TAG}_fs_p$P.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/stamps_${TAG}_fs_p$P.txt; exit 1; }
  echo "=== fs P=$P"; grep -A14 "== fs" $OUT/stamps_${TAG}_fs_p$P.txt
done
fi
