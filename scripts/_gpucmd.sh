set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -k "ppo_update or mopg" > gpurun_out/t_upd.log 2>&1 || { tail -40 gpurun_out/t_upd.log; exit 1; }
tail -1 gpurun_out/t_upd.log
PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 200 python scripts/stamps.py > gpurun_out/stamps_upd.txt 2>&1; grep -A14 "== mfma" gpurun_out/stamps_upd.txt
STAMP_BLOCK=8 PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 200 python scripts/stamps.py > gpurun_out/stamps_upd8.txt 2>&1; grep -A14 "== mfma" gpurun_out/stamps_upd8.txt
bash scripts/bench_prof.sh upd3 | head -4
