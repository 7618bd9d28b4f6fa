# A/B variants of one source without stamps: bash scripts/build_var.sh <source.hip> <n>... -> pgmorl_amd/libpgm_var<n>.so
set -e
src=$1; shift
cd "$(dirname "$0")/.."
# (run python -m pgmorl_amd.build once beforehand: parallel invocations of this script must not race on it)
for n in "$@"; do
  mkdir -p pgmorl_amd/build_var$n
  objs=""
  for o in pgmorl_amd/build/*.o; do
    b=$(basename $o)
    if [ "$b" = "$src.o" ]; then
      /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -DPGM_EXP=$n $EXTRA -c pgmorl_amd/csrc/$src -o pgmorl_amd/build_var$n/$b &
      objs="$objs pgmorl_amd/build_var$n/$b"
    else
      objs="$objs $o"
    fi
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o pgmorl_amd/libpgm_var$n.so
  echo pgmorl_amd/libpgm_var$n.so
done
