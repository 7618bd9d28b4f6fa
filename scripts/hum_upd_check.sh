#!/bin/bash
# GPU box: update parity (incl. wide + production), Humanoid P=20 and Walker P=40 bench lines, full-algorithm HV (Hopper).
set -o pipefail
TAG=${1:-hu}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_production.py -k "ppo_update or production" -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/hu_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/hu_tests_$TAG.log | head -20; tail -20 $OUT/hu_tests_$TAG.log; exit 1; }
tail -1 $OUT/hu_tests_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 > $OUT/hu_${TAG}_hum.json 2> $OUT/hu_${TAG}_hum.err || { echo HUM BENCH FAILED; tail -20 $OUT/hu_${TAG}_hum.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/hu_${TAG}_hum.json'));r=d['roofline'];print('Humanoid P=20', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],2),'ms/step upd', round(r['avg_launch_ms'],3), r['kernel'], 'frac', round(r['frac'],3))"
timeout -k 10 400 python scripts/hv_full.py device --env MO-Hopper-v2 --seeds 0 1 2 3 4 --ref profiles/r02_hvfull2_oracle_hopper.json --out $OUT/r02_hvfull2_hopper.json > $OUT/hvfull2_$TAG.log 2>&1 || { echo HV FAILED; tail -20 $OUT/hvfull2_$TAG.log; exit 1; }
tail -3 $OUT/hvfull2_$TAG.log
