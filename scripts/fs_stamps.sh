#!/bin/bash
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
for P in 5 20; do
  P=$P STAMP_BLOCK=1 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/stamps_${TAG:-r04g}_fs_p$P.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/stamps_${TAG:-r04g}_fs_p$P.txt; exit 1; }
  echo "=== fs P=$P"; grep -A20 "== fs" $OUT/stamps_${TAG:-r04g}_fs_p$P.txt
done
