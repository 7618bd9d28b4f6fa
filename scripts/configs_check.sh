#!/bin/bash
# GPU box: per-GPU bench lines of the BASELINE configs' per-GPU loads + strong-scaling loads.  Usage: bash scripts/configs_check.sh TAG
set -o pipefail
TAG=${1:-cfg}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-whole-run "$@" > $OUT/bench_${TAG}_$n.json 2> $OUT/bench_${TAG}_$n.err || { echo BENCH $n FAILED; tail -5 $OUT/bench_${TAG}_$n.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${TAG}_$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],2),'ms/step', r['kernel'], round(r['avg_launch_ms'],3),'ms frac', round(r['frac'],3))"
}
run walker_p40 && \
run cheetah_p20 --env-name MO-HalfCheetah-v2 --tasks 20 && \
run hopper3_p27 --env-name MO-Hopper-v3 --tasks 27 && \
run humanoid_p20 --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 && \
run hopper2_p5 --env-name MO-Hopper-v2 --tasks 5 --num-processes 1 && \
run strong20 --scaling strong --tasks 20 && \
run strong10 --scaling strong --tasks 10 && \
run strong5 --scaling strong --tasks 5
