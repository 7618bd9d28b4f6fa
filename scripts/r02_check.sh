#!/bin/bash
# GPU box: parity suite (incl. the production-population tests), smoke, weak + strong bench lines with
# rocprof kernel stats.  Usage: bash scripts/r02_check.sh TAG   (libpgm.so prebuilt in-tree)
set -o pipefail
TAG=${1:-r02}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR)" $OUT/gpu_tests_$TAG.log | head -20; tail -30 $OUT/gpu_tests_$TAG.log; exit 1; }
tail -1 $OUT/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke_$TAG.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo BENCH FAILED; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
for P in 40 20 10 5; do
  timeout -k 10 300 python -u bench.py --scaling strong --tasks $P --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_${TAG}_strong$P.json 2> $OUT/bench_${TAG}_strong$P.err || { echo STRONG $P FAILED; tail -20 $OUT/bench_${TAG}_strong$P.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${TAG}_strong$P.json'));print('strong P=$P', round(d['value']/1e6,2),'M/s', round(d['ms_per_step'],2),'ms/step upd', round(d['roofline']['avg_launch_ms'],2))"
done
bash scripts/bench_prof.sh $TAG > $OUT/bp_$TAG.txt 2>&1 || { echo PROF FAILED; tail $OUT/bp_$TAG.txt; exit 1; }
bash scripts/bench_prof.sh ${TAG}_p5 --scaling strong --tasks 5 > $OUT/bp_${TAG}_p5.txt 2>&1 || { echo PROF5 FAILED; tail $OUT/bp_${TAG}_p5.txt; exit 1; }
tail -8 $OUT/bp_$TAG.txt
tail -8 $OUT/bp_${TAG}_p5.txt
echo all done
