"""Reduce rocprofv3 --pmc counter_collection CSVs to per-launch HBM bytes per kernel.

FETCH_SIZE (KB) is doubled on gfx950 (MI355X_MICROARCH.md: it reports half the bytes of wide coalesced reads);
WRITE_SIZE (KB) is taken as is.  Usage: pmc_summary.py DIR [bench args]; prints one JSON object.  It records the
update variant the profiled bench launched (its JSON line in DIR/FETCH_SIZE.log: roofline.kernel, the
pgm_ppo_update_variant string) and the hash of that kernel's sources (bench.kernel_source_hash): bench.py quotes the
summary only for the same variant and sources.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_dispatch(d, counter):
    f = glob.glob(f'{d}/{counter}/**/*counter_collection.csv', recursive=True)
    if not f:
        raise SystemExit(f'no counter_collection.csv under {d}/{counter}')
    acc = defaultdict(float)
    names = {}
    for row in csv.DictReader(open(f[0])):
        if row.get('Counter_Name') != counter:
            continue
        k = row['Dispatch_Id']
        acc[k] += float(row['Counter_Value'])
        names[k] = row['Kernel_Name']
    by_kernel = defaultdict(list)
    for k, v in acc.items():
        by_kernel[names[k]].append(v * 1024.0)  # KB -> bytes
    return by_kernel


def main():
    d = sys.argv[1]
    args = sys.argv[2:]

    def opt(name, default):
        return args[args.index(name) + 1] if name in args else default
    fetch, write = per_dispatch(d, 'FETCH_SIZE'), per_dispatch(d, 'WRITE_SIZE')
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(name, [0])) / max(1, len(fetch.get(name, [])))
        w = sum(write.get(name, [0])) / max(1, len(write.get(name, [])))
        kernels[name] = {'launches': len(fetch.get(name, [])), 'fetch_bytes_raw': f, 'fetch_bytes': 2 * f,
                         'write_bytes': w, 'hbm_bytes_per_launch': 2 * f + w}
    # the update kernel of the workload: the one launched most (a second variant can only come from another leg)
    upd = sorted((k for k in kernels if 'ppo_update_' in k), key=lambda k: (-kernels[k]['launches'], k))
    env, P, N = opt('--env-name', 'MO-Walker2d-v2'), opt('--tasks', '40'), opt('--num-processes', '4')
    T, E, M = opt('--num-steps', '2048'), opt('--ppo-epoch', '10'), opt('--num-mini-batch', '32')
    variant = None
    for line in open(os.path.join(d, 'FETCH_SIZE.log')):
        if line.startswith('{'):
            variant = json.loads(line)['roofline']['kernel']
    from bench import kernel_source_hash
    out = {'workload': f'{env}/P{P}/N{N}/T{T}/E{E}/M{M}',
           'variant': variant, 'source_hash': kernel_source_hash(variant),
           'kernel': upd[0] if upd else None,
           'hbm_bytes_per_launch': kernels[upd[0]]['hbm_bytes_per_launch'] if upd else None,
           'method': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, per-dispatch sums; '
                     'FETCH_SIZE x2 (gfx950 correction), KB x 1024',
           'kernels': kernels}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
