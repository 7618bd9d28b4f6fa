#!/bin/bash
# GPU box: the device side of the full-algorithm HV comparison (scripts/hv_full.py) against the committed
# oracle JSONs.  Usage: bash scripts/hv_device.sh
set -o pipefail
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
for E in hopper walker; do
  timeout -k 10 600 python -u scripts/hv_full.py device --ref profiles/r02_hvfull_oracle_$E.json --out $OUT/r02_hvfull_$E.json > $OUT/hvf_dev_$E.log 2>&1 || { echo HV $E FAILED; tail -20 $OUT/hvf_dev_$E.log; exit 1; }
  tail -1 $OUT/hvf_dev_$E.log
done
