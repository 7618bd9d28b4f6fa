set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "wide" --timeout 120 --timeout-method thread > gpurun_out/t_wide.log 2>&1 || { tail -60 gpurun_out/t_wide.log; exit 1; }
tail -8 gpurun_out/t_wide.log
timeout -k 10 300 python -u bench.py --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_hum.json 2> gpurun_out/bench_hum.err || { tail -30 gpurun_out/bench_hum.err; exit 1; }
cat gpurun_out/bench_hum.json
