#!/bin/bash
# GPU box, kernel iteration loop: the update-kernel parity tests, a short bench line, and the phase stamps of the
# update kernels (MODE 2 at Walker P = 40, t16 at P = 20).  Usage: bash scripts/iter_check.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-it}
K=${2:-"ppo_update or production_update or delayed or delay"}
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/it_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR|Error)" $OUT/it_tests_$TAG.log | head -20; tail -30 $OUT/it_tests_$TAG.log; exit 1; }
tail -1 $OUT/it_tests_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 ${BENCH_ARGS} > $OUT/it_bench_$TAG.json 2> $OUT/it_bench_$TAG.err || { echo BENCH FAILED; tail -20 $OUT/it_bench_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/it_bench_$TAG.json')); r=d['roofline']; w=d.get('whole_run') or {}
print('bench', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', r['kernel'], round(r['avg_launch_ms'],3), 'ms frac', round(r['frac'],4))
if w: print('whole run', round(w['value']/1e6,2), 'M/s wall', round(w['wall_s'],2), 's ratio', round(w['vs_iteration_bench'],3), 'host', round(w['boundary_host_s'],3), 'final', w.get('final_s'), 'mopg', round(w['mopg_s'],3))"
if [ -z "$NO_STAMPS" ]; then
  P=40 STAMP_BLOCK=1 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/it_st_${TAG}_mode2.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/it_st_${TAG}_mode2.txt; exit 1; }
  P=20 STAMP_BLOCK=1 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > $OUT/it_st_${TAG}_t16.txt 2>&1 || { echo STAMPS FAILED; tail $OUT/it_st_${TAG}_t16.txt; exit 1; }
  for f in mode2 t16; do echo "=== $f"; sed -n '/== mfma/,/== lanes/p' $OUT/it_st_${TAG}_$f.txt | grep -v "== lanes"; done
fi
