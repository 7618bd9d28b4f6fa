# stamps of the diagnostic variants: bash scripts/exp_stamps.sh <unit> <n>...
set -o pipefail
mkdir -p gpurun_out
unit=$1; shift
for n in "$@"; do
  echo "=== exp $n"
  ENV=${ENV:-MO-Humanoid-v2} PGM_LIB=pgmorl_amd/libpgm_exp$n.so timeout -k 10 200 python -u scripts/stamps.py > gpurun_out/stamps_exp$n.txt 2>&1 || { tail -20 gpurun_out/stamps_exp$n.txt; exit 1; }
  sed -n "/== $unit/,/^==/p" gpurun_out/stamps_exp$n.txt
done
