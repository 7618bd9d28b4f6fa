#!/bin/bash
# r05b: NS = 6, R = 3 feature-split update (two per CU) at Walker P = 40: parity, then the update time at T = 2304
# (mb = 288 = 16 x 6 x 3) against MODE 2 at T = 2048 and T = 2304.
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fs.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r05b_fs_tests.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/r05b_fs_tests.log | head; tail -30 $OUT/r05b_fs_tests.log; exit 1; }
tail -1 $OUT/r05b_fs_tests.log
run() { tag=$1; shift; timeout -k 10 300 env "$@" > $OUT/r05b_$tag.json 2> $OUT/r05b_$tag.err || { echo BENCH $tag FAILED; tail -20 $OUT/r05b_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r05b_$tag.json'));r=d['roofline'];print('$tag', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],3),'ms/step', r['kernel'], round(r['avg_launch_ms'],3),'ms frac', round(r['frac'],3))"; }
B="python -u bench.py --no-cpu-baseline --no-whole-run --steps 10 --warmup 2"
run mode2_t2048 $B && run fs6_t2304 $B --num-steps 2304 && run mode2_t2304 PGM_UPDATE_KERNEL=mfma $B --num-steps 2304
