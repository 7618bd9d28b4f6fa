#!/bin/bash
# GPU box: full GPU suite + smoke after the two-workgroups-per-CU feature-split placement, the per-config bench lines,
# the device side of the 20-seed Hopper-v3 HV comparison.
set -o pipefail
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_r04s.log 2>&1 || { grep -E "(FAILED|ERROR)" $OUT/gpu_tests_r04s.log | head; tail -30 $OUT/gpu_tests_r04s.log; exit 1; }
tail -1 $OUT/gpu_tests_r04s.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r04s.log 2>&1 || { tail -20 $OUT/smoke_r04s.log; exit 1; }
echo smoke ok
bash scripts/configs_check.sh r04s || exit 1
timeout -k 10 600 python -u scripts/hv_full.py device --ref profiles/r04_hvfull_oracle_hopper3.json --out gpurun_out/r04_hvfull_hopper3.json > gpurun_out/hv_r04s_hopper3.log 2>&1 || { tail -5 gpurun_out/hv_r04s_hopper3.log; exit 1; }
tail -c 600 gpurun_out/hv_r04s_hopper3.log
