"""Reduce the SQ counter passes of scripts/sq_counters.sh to per-launch figures for the update kernel.

Units (MI355X_MICROARCH.md, PMC table): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* / SQ_BUSY_CYCLES count
quad-cycles (x4 = shader cycles); SQ_VALU_MFMA_BUSY_CYCLES counts cycles; GRBM_GUI_ACTIVE is summed over the 8
XCDs, so the effective clock is GRBM_GUI_ACTIVE / 8 / kernel time.  WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
~ WAVE_CYCLES (disjoint), so their shares are where a wave's lifetime goes.
Usage: sq_summary.py DIR [bench args]; prints one JSON object.  Measurement tool, not product code.
"""
import csv
import os
import glob
import json
import sys
from collections import defaultdict


KFILTER = os.environ.get('SQ_KERNEL', 'ppo_update')  # kernel-name substring (e.g. rollout_lane for the rollout)


def load(d):
    per = defaultdict(lambda: defaultdict(float))  # (pass, dispatch) -> counter -> value
    meta = {}
    for f in sorted(glob.glob(f'{d}/g*/**/*counter_collection.csv', recursive=True)):
        gp = f[len(d):].split('/')[1]
        for row in csv.DictReader(open(f)):
            if KFILTER not in row['Kernel_Name']:
                continue
            key = (gp, row['Dispatch_Id'])
            per[key][row['Counter_Name']] += float(row['Counter_Value'])
            meta[key] = (row['Kernel_Name'], int(row['Grid_Size']), int(row['Workgroup_Size']),
                         int(row.get('VGPR_Count') or 0), int(row.get('Accum_VGPR_Count') or 0),
                         int(row.get('LDS_Block_Size') or 0), int(row['End_Timestamp']) - int(row['Start_Timestamp']))
    if not per:
        raise SystemExit(f'no {KFILTER} dispatches under {d}')
    # average every counter over the dispatches of its pass
    sums, counts, dur = defaultdict(float), defaultdict(int), []
    for key, cs in per.items():
        for c, v in cs.items():
            sums[c] += v
            counts[c] += 1
        dur.append(meta[key][-1])
    avg = {c: sums[c] / counts[c] for c in sums}
    name, grid, wg, vgpr, agpr, lds, _ = next(iter(meta.values()))
    return avg, name, grid, wg, vgpr, agpr, lds, sum(dur) / len(dur)


def main():
    d = sys.argv[1]
    args = sys.argv[2:]

    def opt(name, default):
        return args[args.index(name) + 1] if name in args else default
    c, name, grid, wg, vgpr, agpr, lds, ns = load(d)
    waves = c.get('SQ_WAVES', 0.0)
    wave_cyc = 4.0 * c.get('SQ_WAVE_CYCLES', 0.0)
    env, P, N = opt('--env-name', 'MO-Walker2d-v2'), opt('--tasks', '40'), opt('--num-processes', '4')
    T, E, M = opt('--num-steps', '2048'), opt('--ppo-epoch', '10'), opt('--num-mini-batch', '32')
    variant = None  # the launcher's own name of the profiled update (the bench line of pass 1)
    try:
        for line in open(os.path.join(d, 'g1.log')):
            if line.startswith('{'):
                variant = json.loads(line)['roofline']['kernel']
    except (OSError, ValueError, KeyError):
        pass
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_source_hash
    out = {'workload': f'{env}/P{P}/N{N}/T{T}/E{E}/M{M}', 'variant': variant,
           'source_hash': kernel_source_hash(variant) if KFILTER == 'ppo_update' else None,
           'kernel': name, 'grid_threads': grid, 'workgroup': wg, 'vgpr': vgpr, 'agpr': agpr, 'lds_bytes': lds,
           'kernel_ns_profiled': ns, 'counters_per_launch': c,
           'method': 'rocprofv3 --pmc, 2 passes (8 SQ + GRBM / 8 SQ), --kernel-trace only; per-dispatch sums '
                     f'averaged over the {KFILTER} dispatches of each pass'}
    if waves:
        out['waves'] = waves
        out['wave_lifetime_cycles'] = wave_cyc / waves
        out['per_wave'] = {k: c[f'SQ_INSTS_{k}'] / waves for k in ('VALU', 'MFMA', 'LDS', 'SALU')
                           if f'SQ_INSTS_{k}' in c}
    if 'GRBM_GUI_ACTIVE' in c and ns:
        out['clock_ghz'] = c['GRBM_GUI_ACTIVE'] / 8.0 / ns
    if wave_cyc:
        shares = {}
        for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_LDS',
                  'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_MISC'):
            if k in c:
                shares[k] = 4.0 * c[k] / wave_cyc
        out['share_of_wave_cycles'] = shares
        out['wait_any_share'] = shares.get('SQ_WAIT_ANY')
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in c:
            # one wave per SIMD in these kernels (256-thread WGs, one WG per CU): the MFMA pipe's busy share of
            # the SIMD's wave lifetime
            out['mfma_busy_share'] = c['SQ_VALU_MFMA_BUSY_CYCLES'] / wave_cyc
    if 'SQ_LDS_BANK_CONFLICT' in c and 'SQ_ACTIVE_INST_LDS' in c and c['SQ_ACTIVE_INST_LDS']:
        out['lds_bank_conflict_per_active_lds'] = c['SQ_LDS_BANK_CONFLICT'] / c['SQ_ACTIVE_INST_LDS']
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
