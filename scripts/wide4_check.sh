#!/bin/bash
# GPU box: wide (Humanoid) update at NS = 4 (default) and NS = 2 (A/B): parity + bench lines + stamps.
set -o pipefail
OUT=$(pwd)/gpurun_out
mkdir -p $OUT
TAG=${1:-w4}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "wide" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t_wide4_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $OUT/t_wide4_$TAG.log | tail -30; exit 1; }
tail -1 $OUT/t_wide4_$TAG.log
PGM_UPDATE_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "wide" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t_wide2_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $OUT/t_wide2_$TAG.log | tail -30; exit 1; }
tail -1 $OUT/t_wide2_$TAG.log
PGM_UPDATE_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "wide" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t_wide1_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $OUT/t_wide1_$TAG.log | tail -30; exit 1; }
tail -1 $OUT/t_wide1_$TAG.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_production.py -x -q -k "update and Humanoid" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_wideprod_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" $OUT/t_wideprod_$TAG.log | tail -30; exit 1; }
tail -1 $OUT/t_wideprod_$TAG.log
for V in 4 2; do
PGM_UPDATE_SPLIT=$V timeout -k 10 300 python -u bench.py --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_hum_${TAG}_v$V.json 2> $OUT/bench_hum_${TAG}_v$V.err || { tail -30 $OUT/bench_hum_${TAG}_v$V.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_hum_${TAG}_v$V.json'));print('split $V', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],2),'ms/step upd', round(d['roofline']['avg_launch_ms'],2), 'frac', round(d['roofline']['frac'],3))"
done
ENV=MO-Humanoid-v2 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 200 python -u scripts/stamps.py > $OUT/stamps_hum_$TAG.txt 2>&1 || { tail -30 $OUT/stamps_hum_$TAG.txt; exit 1; }
sed -n '/== wupd/,$p' $OUT/stamps_hum_$TAG.txt
