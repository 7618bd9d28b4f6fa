#!/bin/bash
# GPU box: phase stamps (libpgm_stamps.so) of the update kernels at their headline loads: MODE 2 (Walker P=40),
# t16 (Walker P=20), wide (Humanoid P=20), plus the rollouts.  Usage: bash scripts/stamps_all.sh TAG
set -o pipefail
TAG=${1:-st}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
P=40 STAMP_BLOCK=1 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/stamps_${TAG}_mode2.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/stamps_${TAG}_mode2.txt; exit 1; }
P=20 STAMP_BLOCK=1 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/stamps_${TAG}_t16.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/stamps_${TAG}_t16.txt; exit 1; }
ENV=MO-Humanoid-v2 P=20 STAMP_BLOCK=1 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 200 python scripts/stamps.py > $OUT/stamps_${TAG}_wide.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/stamps_${TAG}_wide.txt; exit 1; }
for f in mode2 t16 wide; do echo "=== $f"; grep -A20 -E "== (mfma|wupd|wide|lanes)" $OUT/stamps_${TAG}_$f.txt; done
