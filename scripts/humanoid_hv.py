"""Config 4's hypervolume on the device: SynthMO-Humanoid, pop = 20 per GPU (the 160-task config sharded over 8),
N = 8, T = 2048, gamma 0.99, eval_num 6 (scripts/humanoid-v2.py:37-45), trained iteration after iteration with the
reference's update schedule; after every iteration the EP over every offspring so far (morl/ep.py:23-31, which drops
points with a negative objective: morl/utils.py:37) and its HV (ref point 0).

Why this exists: the energy objective is 3 - 4 sum(ctrl^2) + 3 with ctrl clipped to +-0.4 (environments/humanoid.py:34,
17 actuators), so a freshly initialised policy (std 1: |a| > 0.4 almost always) scores about 6 - 4 * 17 * 0.16 < 0 per
step and an untrained population has an EMPTY Pareto archive (HV 0).  The budget at which training first puts offspring
into the archive is measured here.  The fp64 CPU oracle cannot be run at this size (a 376-input policy, 8 envs x 2,048
steps per iteration per task), so this HV is device-only: no device-vs-oracle comparison exists for config 4.

    python scripts/humanoid_hv.py --iters 200 --out profiles/r04_humanoid_hv.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pgmorl_amd import pareto  # noqa: E402
from pgmorl_amd.policy import new_policy  # noqa: E402
from pgmorl_amd.runtime import TaskBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--tasks', type=int, default=20)
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    env, P, N, T = 'MO-Humanoid-v2', a.tasks, 8, 2048
    tb = TaskBatch(env, P, num_processes=N, num_steps=T, gamma=0.99, eval_num=6, seed=a.seed)
    torch.manual_seed(a.seed)
    w = np.linspace(0, 1, 160)[:P]  # rank 0's block of the 160-task weight grid (delta 1/159)
    for p in range(P):
        tb.set_task(p, new_policy(tb.O, tb.A, tb.K).state_dict(), {}, None, [w[p], 1 - w[p]])
    tb.env_reset()
    total = int(8e6) // T // N  # scripts/humanoid-v2.py: 8e6 env steps per task
    objs_all, rows = [], []
    t0 = time.time()
    for j in range(a.iters):
        tb.iteration(j, 3e-4 * (1 - j / total), carry=j > 0)
        o = tb.objs.cpu().numpy().copy()
        objs_all.append(o)
        allo = np.concatenate(objs_all)
        idx = pareto.get_ep_indices(allo)
        hv = pareto.compute_hypervolume(allo[idx]) if len(idx) else 0.0
        rows.append({'iter': j + 1, 'env_steps_per_task': (j + 1) * T * N, 'ep_size': int(len(idx)), 'hv': float(hv),
                     'objs_mean': o.mean(0).tolist(), 'objs_max': o.max(0).tolist()})
        if (j + 1) % 10 == 0:
            print(json.dumps(rows[-1]), flush=True)
    tb.check_update()
    first = next((r['iter'] for r in rows if r['ep_size'] > 0), None)
    out = {'env': env, 'tasks': P, 'N': N, 'T': T, 'gamma': 0.99, 'eval_num': 6, 'seed': a.seed, 'wall_s': time.time() - t0,
           'first_nonempty_ep_iter': first, 'per_iter': rows,
           'note': 'device-only (perf-mode RNG); EP over every offspring objective so far, non-negative points only '
                   '(morl/utils.py:37), HV vs the origin'}
    with open(a.out, 'w') as f:
        json.dump(out, f)
    print(json.dumps({k: v for k, v in out.items() if k != 'per_iter'}))


if __name__ == '__main__':
    main()
