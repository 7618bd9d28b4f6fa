#!/bin/bash
# GPU box A/B: bench lines of several libraries, alternating, ROUNDS times each, for each workload.
#   bash scripts/ab.sh TAG "libpgm libpgm_prev" ROUNDS "bench args 1" ["bench args 2" ...]
# prints one line per run (lib, workload, env-steps/s, ms/step, update kernel, update ms, frac) -> gpurun_out/ab_TAG.txt
set -o pipefail
TAG=$1; LIBS=$2; ROUNDS=$3; shift 3
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
for args in "$@"; do
  for r in $(seq $ROUNDS); do
    for lib in $LIBS; do
      PGM_LIB=pgmorl_amd/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-whole-run --steps 10 --warmup 2 $args \
          > $OUT/ab_${TAG}_cur.json 2> $OUT/ab_${TAG}_cur.err || { echo "BENCH $lib $args FAILED"; tail -20 $OUT/ab_${TAG}_cur.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/ab_${TAG}_cur.json'));r=d['roofline'];print('$lib', '[$args]', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],3),'ms/step', r['kernel'], round(r['avg_launch_ms'],3),'ms frac', round(r['frac'],3))" | tee -a $OUT/ab_$TAG.txt
    done
  done
done
