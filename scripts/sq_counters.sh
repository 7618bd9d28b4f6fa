#!/bin/bash
# SQ counters of the update kernel (one bench step), one rocprofv3 --pmc pass per counter group.
# Usage: scripts/sq_counters.sh TAG  -> gpurun_out/sq_TAG/<group>/...
set -o pipefail
TAG=${1:-run}; shift
R=$(pwd)
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace -d $OUT/g$i -o g$i --output-format csv -- \
      python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-whole-run "$@" > $OUT/g$i.log 2>&1 || { echo "group $i failed"; tail -5 $OUT/g$i.log; }
done
python - <<PY
import csv, glob, collections
for f in sorted(glob.glob('$OUT/g*/**/*counter_collection.csv', recursive=True)):
    acc = collections.defaultdict(float)
    for row in csv.DictReader(open(f)):
        if 'ppo_update' in row['Kernel_Name']:
            acc[row['Counter_Name']] += float(row['Counter_Value'])
    for k, v in sorted(acc.items()):
        print(f'{k:28s} {v:.4e}')
PY
