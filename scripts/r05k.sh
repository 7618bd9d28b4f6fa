#!/bin/bash
# r05k: phase stamps of the fs update, compact fragments (libpgm_stamps) vs the previous layout (libpgm_stampsprev),
# Walker P = 5 (NS 16) and P = 40 (NS 6), HalfCheetah P = 20 (NS 8)
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
for cfg in "MO-Walker2d-v2 5" "MO-Walker2d-v2 40" "MO-HalfCheetah-v2 20"; do
  set -- $cfg
  for lib in stamps stampsprev; do
    ENV=$1 P=$2 STAMP_BLOCK=0 PGM_LIB=pgmorl_amd/libpgm_$lib.so timeout -k 10 120 python scripts/stamps.py > $OUT/r05k_${lib}_$1_$2.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/r05k_${lib}_$1_$2.txt; exit 1; }
    echo "=== $lib $1 P=$2"; grep -A20 "== fs" $OUT/r05k_${lib}_$1_$2.txt
  done
done
