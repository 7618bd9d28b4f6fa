#!/bin/bash
# HBM traffic of the dominant kernel from PMC counters (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE in
# separate passes (they do not fit one TCC pass), kernel-trace only, no runtime/sys traces.
# Usage: scripts/pmc.sh TAG [bench args]   -> gpurun_out/pmc_TAG/{fetch,write}/..., gpurun_out/pmc_TAG.json
set -o pipefail
TAG=${1:-run}; shift
R=$(pwd)
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace -d $OUT/$C -o $C --output-format csv -- \
      python $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-whole-run "$@" > $OUT/$C.log 2>&1 \
      || { echo "PMC $C FAILED"; tail -20 $OUT/$C.log; exit 1; }
done
python $R/scripts/pmc_summary.py $OUT "$@" > $R/gpurun_out/pmc_$TAG.json && cat $R/gpurun_out/pmc_$TAG.json
