#!/bin/bash
# GPU box: the device side of the full-algorithm HV comparison (scripts/hv_full.py) against a committed oracle JSON.
# Usage: bash scripts/hv_device.sh TAG ORACLE_JSON [ORACLE_JSON ...]   -> gpurun_out/<TAG>_<env>.json
set -o pipefail
TAG=${1:-hv}; shift
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
for REF in "$@"; do
  E=$(basename $REF .json | sed 's/.*oracle_//')
  timeout -k 10 600 python -u scripts/hv_full.py device --ref $REF --out $OUT/${TAG}_$E.json > $OUT/${TAG}_$E.log 2>&1 || { echo HV $E FAILED; tail -20 $OUT/${TAG}_$E.log; exit 1; }
  tail -1 $OUT/${TAG}_$E.log
done
