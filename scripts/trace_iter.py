"""Timeline of the last MOPG iteration in a rocprofv3 --kernel-trace CSV (bench.py run): every kernel between the
last two update-kernel launches, with its stream, start offset, duration and the idle gap before it on its stream.
Shows what besides the rollout and the update sits on the iteration's critical path.

    python scripts/trace_iter.py gpurun_out/prof_TAG/..._kernel_trace.csv
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    upd = [i for i, r in enumerate(rows) if 'ppo_update_' in r['Kernel_Name']]
    if len(upd) < 2:
        raise SystemExit('need two update launches in the trace')
    a, b = upd[-2], upd[-1]
    t0 = int(rows[a]['End_Timestamp'])
    last_end = {}
    print(f"iteration: update end -> next update end = {(int(rows[b]['End_Timestamp']) - t0) / 1e3:.1f} us")
    busy = 0
    for r in rows[a + 1:b + 1]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        q = r['Queue_Id']
        gap = (s - last_end.get(q, t0)) / 1e3
        last_end[q] = e
        name = r['Kernel_Name'].split('(')[0].replace('void ', '')[:58]
        print(f'  q{q:>2} +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  {name}')
        busy += e - s


if __name__ == '__main__':
    main()
