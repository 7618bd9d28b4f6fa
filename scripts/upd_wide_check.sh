set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "wide" --timeout 120 --timeout-method thread > gpurun_out/t_wide.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/t_wide.log | tail -30; exit 1; }
tail -3 gpurun_out/t_wide.log
PGM_UPDATE_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "wide" --timeout 120 --timeout-method thread > gpurun_out/t_wide1.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/t_wide1.log | tail -30; exit 1; }
tail -1 gpurun_out/t_wide1.log
timeout -k 10 300 python -u bench.py --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_hum.json 2> gpurun_out/bench_hum.err || { tail -30 gpurun_out/bench_hum.err; exit 1; }
cat gpurun_out/bench_hum.json
ENV=MO-Humanoid-v2 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 200 python -u scripts/stamps.py > gpurun_out/stamps_hum.txt 2>&1 || { tail -30 gpurun_out/stamps_hum.txt; exit 1; }
sed -n '/== wupd/,$p' gpurun_out/stamps_hum.txt
