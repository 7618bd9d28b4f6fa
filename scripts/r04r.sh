#!/bin/bash
# GPU box: the feature-split update with two workgroups per CU (R <= 2 where 16 NS ceil(P/8) > CUs): parity (fs,
# exchange delays, production), then A/B bench lines dual vs one per CU (PGM_FS_DUAL=0).
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fs.py tests/test_gpu_exchange.py tests/test_gpu_production.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r04r_tests.log 2>&1 || { tail -30 $OUT/r04r_tests.log; exit 1; }
tail -2 $OUT/r04r_tests.log
run() { local n=$1 e=$2; shift 2
  env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-whole-run --no-strong "$@" > $OUT/ab_r04r_$n.json 2> $OUT/ab_r04r_$n.err || { echo BENCH $n FAILED; tail -5 $OUT/ab_r04r_$n.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/ab_r04r_$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],3),'ms/step', r['kernel'], round(r['avg_launch_ms'],3),'ms frac', round(r['frac'],3))"; }
run p20_dual '' --scaling strong --tasks 20 && run p20_one PGM_FS_DUAL=0 --scaling strong --tasks 20 && \
run p10_dual '' --scaling strong --tasks 10 && run p10_one PGM_FS_DUAL=0 --scaling strong --tasks 10 && \
run cheetah_p20_dual '' --env-name MO-HalfCheetah-v2 --tasks 20 && run cheetah_p20_one PGM_FS_DUAL=0 --env-name MO-HalfCheetah-v2 --tasks 20 && \
run hopper3_p27_dual '' --env-name MO-Hopper-v3 --tasks 27 && run hopper3_p27_one PGM_FS_DUAL=0 --env-name MO-Hopper-v3 --tasks 27 && \
run p5 '' --scaling strong --tasks 5 && run p40 '' --scaling strong --tasks 40
