#!/bin/bash
# r05l: compact fs fragments with launch-fixed owner / head-block indices: fs GPU tests, A/B vs the previous layout,
# phase stamps at Walker P = 5 / 40
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fs.py tests/test_gpu_exchange.py tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r05l_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/r05l_gpu_tests.log; exit 1; }
tail -1 $OUT/r05l_gpu_tests.log
rm -f $OUT/ab_r05l.txt
bash scripts/ab.sh r05l "libpgm libpgm_prev" 2 "" "--env-name MO-HalfCheetah-v2 --tasks 20" "--tasks 5" > /dev/null || exit 1
cat $OUT/ab_r05l.txt
for cfg in "MO-Walker2d-v2 5" "MO-Walker2d-v2 40"; do
  set -- $cfg
  for lib in stamps; do
    ENV=$1 P=$2 STAMP_BLOCK=0 PGM_LIB=pgmorl_amd/libpgm_$lib.so timeout -k 10 120 python scripts/stamps.py > $OUT/r05l_${lib}_$1_$2.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/r05l_${lib}_$1_$2.txt; exit 1; }
    echo "=== $lib $1 P=$2"; grep -A20 "== fs" $OUT/r05l_${lib}_$1_$2.txt
  done
done
