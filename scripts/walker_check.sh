set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "ppo_update or update" --timeout 120 --timeout-method thread > gpurun_out/t_upd.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/t_upd.log | tail -30; exit 1; }
tail -1 gpurun_out/t_upd.log
PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 200 python -u scripts/stamps.py > gpurun_out/stamps_walker.txt 2>&1 || { tail -20 gpurun_out/stamps_walker.txt; exit 1; }
sed -n "/== mfma/,/== lanes/p" gpurun_out/stamps_walker.txt | head -3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_walker.json 2> gpurun_out/bench_walker.err || { tail -30 gpurun_out/bench_walker.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_walker.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
