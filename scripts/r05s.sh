#!/bin/bash
# r05s: phase stamps of an ACTOR workgroup (block 8: task 0, actor tower, part 0) beside the critic (block 0)
set -o pipefail
for cfg in "MO-Walker2d-v2 5" "MO-HalfCheetah-v2 20" "MO-Walker2d-v2 40"; do
  set -- $cfg
  for B in 0 8; do
    ENV=$1 P=$2 STAMP_BLOCK=$B PGM_LIB=pgmorl_amd/libpgm_stamps.so timeout -k 10 120 python scripts/stamps.py > gpurun_out/r05s_stamps_$1_$2_b$B.txt 2>&1 || { echo STAMPS FAILED; tail gpurun_out/r05s_stamps_$1_$2_b$B.txt; exit 1; }
  done
  python - $1 $2 <<'PY'
import re, sys
env, P = sys.argv[1], sys.argv[2]
def read(b):
    t = open(f'gpurun_out/r05s_stamps_{env}_{P}_b{b}.txt').read()
    t = t[t.index('== fs'):]
    return {int(m.group(1)): (m.group(2).strip(), int(m.group(3))) for m in re.finditer(r'phase\s+(\d+) (.{22,40}?)\s+(\d+) cycles', t)}
c, a = read(0), read(8)
print(f'=== {env} P={P}: phase, critic (block 0), actor (block 8)')
for k in sorted(c):
    print(f'  {k:2d} {c[k][0]:22s} {c[k][1]:7d} {a.get(k, ("", 0))[1]:7d}')
print('  total', sum(v[1] for v in c.values()), sum(v[1] for v in a.values()))
PY
done
