#!/bin/bash
# GPU box: the device side of every committed oracle HV run (scripts/hv_full.py).  Usage: bash scripts/hv_device.sh TAG
set -o pipefail
TAG=${1:-r04}
for env in hopper hopper3; do
  ref=profiles/${TAG}_hvfull_oracle_${env}.json
  [ -f $ref ] || continue
  timeout -k 10 600 python -u scripts/hv_full.py device --ref $ref --out gpurun_out/${TAG}_hvfull_${env}.json > gpurun_out/hv_${TAG}_${env}.log 2>&1 || { echo HV $env FAILED; tail -5 gpurun_out/hv_${TAG}_${env}.log; exit 1; }
  tail -c 400 gpurun_out/hv_${TAG}_${env}.log; echo
done
