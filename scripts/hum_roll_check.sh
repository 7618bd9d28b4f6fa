#!/bin/bash
# GPU box: Humanoid rollout / eval / update parity (kernel + production tests), then the Humanoid P=20 bench line.
set -o pipefail
TAG=${1:-hr}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_production.py tests/test_gpu_golden.py -k "Humanoid or wide or production" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/hr_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/hr_tests_$TAG.log | head -20; tail -20 $OUT/hr_tests_$TAG.log; exit 1; }
tail -1 $OUT/hr_tests_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 > $OUT/hr_${TAG}_hum.json 2> $OUT/hr_${TAG}_hum.err || { echo HUM BENCH FAILED; tail -20 $OUT/hr_${TAG}_hum.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/hr_${TAG}_hum.json'));r=d['roofline'];print('Humanoid P=20', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],2),'ms/step upd', round(r['avg_launch_ms'],3), r['kernel'], 'frac', round(r['frac'],3))"
