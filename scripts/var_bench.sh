#!/bin/bash
# GPU box: bench the A/B variant libraries (scripts/build_var.sh).  Usage: bash scripts/var_bench.sh TAG "lib:tasks" ...
set -o pipefail
TAG=$1; shift
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
for spec in "$@"; do
  lib=${spec%%:*}; P=${spec##*:}
  PGM_LIB=pgmorl_amd/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --scaling strong --tasks $P --steps ${STEPS:-10} --warmup 2 $BENCH_ARGS > $OUT/var_${TAG}_${lib}_p$P.json 2> $OUT/var_${TAG}_${lib}_p$P.err || { echo BENCH $spec FAILED; tail -20 $OUT/var_${TAG}_${lib}_p$P.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/var_${TAG}_${lib}_p$P.json'));r=d['roofline'];print('$lib P=$P', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],3),'ms/step upd', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],3))"
done
