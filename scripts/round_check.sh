#!/bin/bash
# GPU box routine: the -m gpu parity suite, smoke(), the default bench line (iteration bench + whole run +
# cpu_baseline), and rocprofv3 kernel stats of the iteration bench.  libpgm.so is prebuilt in-tree.
# Usage: bash scripts/round_check.sh TAG [--no-tests] [bench args]
set -o pipefail
TAG=${1:-run}; shift
TESTS=1
if [ "$1" = "--no-tests" ]; then TESTS=0; shift; fi
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
      > $OUT/gpu_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR)" $OUT/gpu_tests_$TAG.log | head -20; tail -30 $OUT/gpu_tests_$TAG.log; exit 1; }
  tail -1 $OUT/gpu_tests_$TAG.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke_$TAG.log; exit 1; }
  echo smoke ok
fi
timeout -k 10 600 python -u bench.py "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo BENCH FAILED; tail -20 $OUT/bench_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench_$TAG.json')); r=d['roofline']; w=d.get('whole_run') or {}; c=d.get('cpu_baseline') or {}
print('bench', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', r['kernel'], round(r['avg_launch_ms'],3), 'ms frac', round(r['frac'],4))
print('whole run', round(w.get('value',0)/1e6,2), 'M/s wall', round(w.get('wall_s',0),2), 's ratio', round(w.get('vs_iteration_bench',0),3), 'host share', round(w.get('host_share',0),3))
print('cpu', c.get('value'), c.get('cores'), 'vs 96vCPU', d.get('vs_96vcpu_extrapolated'))"
bash scripts/bench_prof.sh $TAG "$@" > $OUT/bp_$TAG.txt 2>&1 || { echo PROF FAILED; tail $OUT/bp_$TAG.txt; exit 1; }
tail -8 $OUT/bp_$TAG.txt
echo all done
