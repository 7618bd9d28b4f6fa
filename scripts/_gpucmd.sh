set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
bash scripts/bench_prof.sh v21 > gpurun_out/bp.txt; head -5 gpurun_out/bp.txt
