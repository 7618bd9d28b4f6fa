#!/bin/bash
# GPU box: full parity suite, smoke, headline bench (with cpu_baseline), rocprof kernel stats, PMC traffic,
# Humanoid bench + kernel stats.  Usage: bash scripts/final_check.sh TAG   (libpgm.so prebuilt in-tree)
set -o pipefail
TAG=${1:-final}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "^(FAILED|ERROR)" $OUT/gpu_tests_$TAG.log | head; tail -5 $OUT/gpu_tests_$TAG.log; exit 1; }
tail -1 $OUT/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke_$TAG.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo BENCH FAILED; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
bash scripts/bench_prof.sh $TAG > $OUT/bp_$TAG.txt 2>&1 || { echo PROF FAILED; tail $OUT/bp_$TAG.txt; exit 1; }
bash scripts/pmc.sh $TAG > $OUT/pmc_$TAG.txt 2>&1 || { echo PMC FAILED; tail $OUT/pmc_$TAG.txt; exit 1; }
bash scripts/bench_prof.sh ${TAG}h --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 > $OUT/bp_${TAG}h.txt 2>&1 || { echo HPROF FAILED; tail $OUT/bp_${TAG}h.txt; exit 1; }
tail -8 $OUT/bp_$TAG.txt
echo all done
