set -o pipefail
PGM_UPDATE_KERNEL=fs timeout -k 10 200 python -u scripts/diag_fs.py MO-Hopper-v2 5 1 64 > gpurun_out/diag1.txt 2>&1; echo rc=$?; tail -30 gpurun_out/diag1.txt
