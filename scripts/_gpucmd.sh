set -o pipefail
mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tests/hip/multisum_check.hip -o gpurun_out/multisum_check && timeout -k 5 60 gpurun_out/multisum_check || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "rollout or eval or mopg" > gpurun_out/t_lanes.log 2>&1 || { tail -40 gpurun_out/t_lanes.log; exit 1; }
tail -3 gpurun_out/t_lanes.log
PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 200 python scripts/stamps.py > gpurun_out/stamps_lanes.txt 2>&1; grep -A12 "== lanes" gpurun_out/stamps_lanes.txt
bash scripts/bench_prof.sh lanes3
