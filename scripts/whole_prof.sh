#!/bin/bash
# GPU box: cProfile of the whole run (scripts/prof_whole.py) + a kernel trace of it (device busy vs wall).
# Usage: bash scripts/whole_prof.sh TAG
set -o pipefail
TAG=${1:-wp}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u scripts/prof_whole.py $OUT/prof_whole_$TAG.txt > $OUT/prof_whole_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_whole_$TAG.log; exit 1; }
tail -1 $OUT/prof_whole_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/ktrace_$TAG -o kt --output-format csv -- python $R/scripts/prof_whole.py /tmp/pw.txt > $OUT/ktrace_$TAG.log 2>&1 || { echo KTRACE FAILED; tail -20 $OUT/ktrace_$TAG.log; exit 1; }
python - <<PY
import csv, glob
f = glob.glob('$OUT/ktrace_$TAG/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in csv.DictReader(open(f)))
# second whole run only (the profiler script runs two): split at the largest gap
gaps = [(rows[i + 1][0] - rows[i][1], i) for i in range(len(rows) - 1)]
big = max(gaps)[1]
rows = rows[big + 1:]
t0, t1 = rows[0][0], max(r[1] for r in rows)
busy, end = 0, t0
for s, e, n in rows:
    if e > end:
        busy += e - max(s, end)
        end = e
print(f'second run: {len(rows)} kernels, span {(t1 - t0) / 1e9:.3f} s, device busy {busy / 1e9:.3f} s ({100 * busy / (t1 - t0):.1f}%)')
gl = sorted(((rows[i + 1][0] - rows[i][1]) / 1e6, i) for i in range(len(rows) - 1))[-12:]
for g, i in gl:
    print(f'gap {g:.2f} ms after {rows[i][2][:50]} -> {rows[i + 1][2][:50]}')
PY
