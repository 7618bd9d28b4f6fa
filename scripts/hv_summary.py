"""Collect the device-vs-oracle HV@budget comparisons (scripts/hv_budget.py outputs) into
profiles/r01_hv_budget.json, the file bench.py quotes.  Usage: python scripts/hv_summary.py profiles/r01_hv_device_*.json"""
import json
import os
import sys

import numpy as np

runs = []
for path in sys.argv[1:]:
    d = json.load(open(path))
    v = d['vs_oracle']
    runs.append({'env': d['env'], 'tasks': d['tasks'], 'iters': d['iters'], 'N': d['N'], 'seed': d['seed'],
                 'budget_env_steps': d['budget_env_steps'], 'hv_device': v['hv_device'], 'hv_oracle': v['hv_oracle'],
                 'hv_rel_diff': v['hv_rel_diff'], 'ep_size_device': v['ep_size_device'],
                 'ep_size_oracle': v['ep_size_oracle'], 'device_wall_s': d['wall_s'],
                 'oracle_wall_s': v['oracle_wall_s'], 'source': os.path.basename(path)})
summary = {}
for env in sorted({r['env'] for r in runs}):
    rs = [r for r in runs if r['env'] == env]
    hd, ho = np.mean([r['hv_device'] for r in rs]), np.mean([r['hv_oracle'] for r in rs])
    summary[env] = {'seeds': len(rs), 'mean_hv_device': hd, 'mean_hv_oracle': ho, 'mean_hv_rel_diff': (hd - ho) / ho,
                    'max_abs_seed_rel_diff': max(abs(r['hv_rel_diff']) for r in rs)}
out = {'what': 'HV of the warm-up-stage EP at an equal env-step budget, device (fp32, MI355X) vs fp64 oracle, '
               'same initial policies and the reference RNG draws (scripts/hv_budget.py)', 'runs': runs,
       'summary': summary}
json.dump(out, open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles',
                                 'r01_hv_budget.json'), 'w'), indent=1)
print(json.dumps(summary, indent=1))
