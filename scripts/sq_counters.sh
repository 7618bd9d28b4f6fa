#!/bin/bash
# SQ counters of the update kernel, one rocprofv3 --pmc pass per counter group (kernel trace only, no
# runtime/sys traces; <= 8 SQ + 2 GRBM counters per pass).  Stops at the first failed pass.
# Usage: scripts/sq_counters.sh TAG [bench args]  -> gpurun_out/sq_TAG/g*/..., gpurun_out/sq_TAG.json
set -o pipefail
TAG=${1:-run}; shift
R=$(pwd)
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT"
i=0
for G in "$G1" "$G2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $G --kernel-trace -d $OUT/g$i -o g$i --output-format csv -- \
      python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-whole-run "$@" > $OUT/g$i.log 2>&1 \
      || { echo "SQ group $i FAILED"; tail -5 $OUT/g$i.log; exit 1; }
done
python $R/scripts/sq_summary.py $OUT "$@" > $R/gpurun_out/sq_$TAG.json && cat $R/gpurun_out/sq_$TAG.json
