#!/bin/bash
# GPU box: t16 single-tile (ONE) variants -- update parity tests, then Walker P=40 with the 8-wave NS=2 t16 kernel
# (PGM_UPDATE_SPLIT=3) vs the default launcher choice, and P=20 (t16 NS=4).  Usage: bash scripts/one_check.sh TAG
set -o pipefail
TAG=${1:-one}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "ppo_update and (t16 or mfma)" -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/one_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/one_tests_$TAG.log | head -20; tail -20 $OUT/one_tests_$TAG.log; exit 1; }
tail -1 $OUT/one_tests_$TAG.log
for cfg in "3 40" "2 40" "4 20" "3 20"; do
  set -- $cfg
  PGM_UPDATE_SPLIT=$1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --scaling strong --tasks $2 --steps 10 --warmup 2 > $OUT/one_${TAG}_s$1_p$2.json 2> $OUT/one_${TAG}_s$1_p$2.err || { echo BENCH $cfg FAILED; tail -20 $OUT/one_${TAG}_s$1_p$2.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/one_${TAG}_s$1_p$2.json'));r=d['roofline'];print('split $1 P=$2', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],2),'ms/step upd', round(r['avg_launch_ms'],3), r['kernel'], 'frac', round(r['frac'],3))"
done
