#!/bin/bash
# r05c: phase stamps of the feature-split update, NS = 6 R = 3 two per CU (Walker P = 40, T = 2304) and NS = 8 R = 2
# two per CU (Walker P = 20), sampled workgroup 0 (task 0, critic, part 0)
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
for cfg in "40 2304" "20 2048"; do
  set -- $cfg
  P=$1 T=$2 STAMP_BLOCK=0 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/r05c_stamps_fs_p$1.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/r05c_stamps_fs_p$1.txt; exit 1; }
  echo "=== fs P=$1 T=$2"; grep -A20 "== fs" $OUT/r05c_stamps_fs_p$1.txt
done
