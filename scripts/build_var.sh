# A/B variant library: libpgm.so with ONE translation unit replaced by another version of it.
#   bash scripts/build_var.sh NAME UNIT.hip VARIANT_SOURCE   -> pgmorl_amd/libpgm_NAME.so
# e.g. bash scripts/build_var.sh prev pgm_ppo_fs.hip <(git show HEAD~1:pgmorl_amd/csrc/pgm_ppo_fs.hip)
# (run python -m pgmorl_amd.build first: the other objects come from pgmorl_amd/build, or $BUILD, e.g.
#  BUILD=pgmorl_amd/build_stamps EXTRA=-DPGM_STAMPS for a phase-stamp variant)
set -e
name=$1; unit=$2; src=$3
cd "$(dirname "$0")/.."
mkdir -p pgmorl_amd/build_var_$name
cp "$src" pgmorl_amd/build_var_$name/$unit
objs=""
for o in ${BUILD:-pgmorl_amd/build}/*.o; do
  b=$(basename $o)
  if [ "$b" = "$unit.o" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I pgmorl_amd/csrc $EXTRA \
        -c pgmorl_amd/build_var_$name/$unit -o pgmorl_amd/build_var_$name/$b
    objs="$objs pgmorl_amd/build_var_$name/$b"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o pgmorl_amd/libpgm_$name.so
echo pgmorl_amd/libpgm_$name.so
