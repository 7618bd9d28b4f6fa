#!/bin/bash
# r05d: the ragged 6-part feature-split update (Walker P = 40 default): full GPU suite, bench lines fs6 vs MODE 2,
# phase stamps of the fs update at P = 40 (NS 6) and P = 20 (NS 8)
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/r05d_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR)" $OUT/r05d_gpu_tests.log | head -20; tail -30 $OUT/r05d_gpu_tests.log; exit 1; }
tail -1 $OUT/r05d_gpu_tests.log
run() { tag=$1; shift; timeout -k 10 300 env "$@" > $OUT/r05d_$tag.json 2> $OUT/r05d_$tag.err || { echo BENCH $tag FAILED; tail -20 $OUT/r05d_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r05d_$tag.json'));r=d['roofline'];print('$tag', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],3),'ms/step', r['kernel'], round(r['avg_launch_ms'],3),'ms frac', round(r['frac'],3))"; }
B="python -u bench.py --no-cpu-baseline --no-whole-run --steps 10 --warmup 2"
run fs6 $B && run mode2 PGM_UPDATE_KERNEL=mfma $B && run fs6b $B && run mode2b PGM_UPDATE_KERNEL=mfma $B || exit 1
for cfg in "40 2048" "20 2048"; do
  set -- $cfg
  P=$1 T=$2 STAMP_BLOCK=0 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/r05d_stamps_fs_p$1.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/r05d_stamps_fs_p$1.txt; exit 1; }
  echo "=== fs P=$1 T=$2"; grep -A20 "== fs" $OUT/r05d_stamps_fs_p$1.txt
done
