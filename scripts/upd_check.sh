#!/bin/bash
# GPU box: update-kernel parity (kernel + production tests), then Walker P=40 / P=20 bench lines.
set -o pipefail
TAG=${1:-upd}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_production.py -k "ppo_update or production" -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/upd_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/upd_tests_$TAG.log | head -20; tail -20 $OUT/upd_tests_$TAG.log; exit 1; }
tail -1 $OUT/upd_tests_$TAG.log
for P in 40 20; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --scaling strong --tasks $P --steps 10 --warmup 2 > $OUT/upd_${TAG}_p$P.json 2> $OUT/upd_${TAG}_p$P.err || { echo BENCH $P FAILED; tail -20 $OUT/upd_${TAG}_p$P.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/upd_${TAG}_p$P.json'));r=d['roofline'];print('P=$P', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],3),'ms/step upd', round(r['avg_launch_ms'],3), r['kernel'], 'frac', round(r['frac'],3))"
done
