#!/bin/bash
set -o pipefail
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
for V in 2 4; do for B in 0 1; do
PGM_UPDATE_SPLIT=$V P=20 STAMP_BLOCK=$B PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/stamps_t16_v${V}_b${B}.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/stamps_t16_v${V}_b${B}.txt; exit 1; }
echo "=== split $V block $B"; grep -A18 "== mfma" $OUT/stamps_t16_v${V}_b${B}.txt
done; done
