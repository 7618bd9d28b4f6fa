#!/bin/bash
# GPU box: MODE-2 single-tile variant -- update parity tests, Walker P=40 bench (default launcher = MODE 2), stamps.
set -o pipefail
TAG=${1:-m2}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "ppo_update and (t16 or mfma)" -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/m2_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/m2_tests_$TAG.log | head -20; tail -20 $OUT/m2_tests_$TAG.log; exit 1; }
tail -1 $OUT/m2_tests_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/m2_${TAG}_p40.json 2> $OUT/m2_${TAG}_p40.err || { echo BENCH FAILED; tail -20 $OUT/m2_${TAG}_p40.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/m2_${TAG}_p40.json'));r=d['roofline'];print('P=40', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],2),'ms/step upd', round(r['avg_launch_ms'],3), r['kernel'], 'frac', round(r['frac'],3))"
PGM_UPDATE_SPLIT=2 P=40 STAMP_BLOCK=1 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/stamps_${TAG}.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/stamps_${TAG}.txt; exit 1; }
grep -A18 "== mfma" $OUT/stamps_${TAG}.txt
