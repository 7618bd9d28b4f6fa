#!/bin/bash
# GPU box: rollout parity + production tests, the fs tests (tagged hop after the slot-size fix), bench lines and stamps.
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_production.py tests/test_gpu_fs.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r04h_tests.log 2>&1 || { tail -30 $OUT/r04h_tests.log; exit 1; }
tail -2 $OUT/r04h_tests.log
bash scripts/fs_ab.sh r04h || exit 1
run() { local n=$1 e=$2; shift 2
  env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-whole-run --no-strong "$@" > $OUT/ab_r04h_$n.json 2> $OUT/ab_r04h_$n.err || { echo BENCH $n FAILED; tail -5 $OUT/ab_r04h_$n.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/ab_r04h_$n.json'));r=d['roofline'];print('$n', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],3),'ms/step', r['kernel'], round(r['avg_launch_ms'],3),'ms frac', round(r['frac'],3))"; }
run p20_ptag PGM_FS_PTAG=1 --scaling strong --tasks 20 || true
P=40 STAMP_BLOCK=1 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/stamps_r04h_p40.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/stamps_r04h_p40.txt; exit 1; }
grep -A8 "== lanes" $OUT/stamps_r04h_p40.txt
