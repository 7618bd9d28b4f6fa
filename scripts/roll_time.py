"""Diagnostic: average time of one rollout launch (pgm_rollout: rollout kernel + critic values) for each library named
on the command line, on the same tasks (PGM_LIB selects the library, one subprocess per library).

    python scripts/roll_time.py pgmorl_amd/libpgm.so pgmorl_amd/libpgm_var44.so [--env MO-Walker2d-v2 --tasks 40]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from pgmorl_amd.policy import new_policy
    from pgmorl_amd.runtime import TaskBatch
    tb = TaskBatch(a.env, a.tasks, num_processes=a.N, num_steps=2048, seed=0)
    torch.manual_seed(0)
    for p in range(a.tasks):
        w = p / max(1, a.tasks - 1)
        wts = [w, 1 - w] if tb.K == 2 else [1.0 / tb.K] * tb.K
        tb.set_task(p, new_policy(tb.O, tb.A, tb.K).state_dict(), {}, None, wts)
    tb.env_reset()
    torch.cuda.synchronize()
    for j in range(3):
        tb.rollout(j, noise=tb.noise)  # the perf-mode path reads drawn noise
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for j in range(a.reps):
        tb.rollout(3 + j, noise=tb.noise)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({'lib': os.environ.get('PGM_LIB', 'default'), 'env': a.env, 'tasks': a.tasks,
                      'rollout_ms': e0.elapsed_time(e1) / a.reps}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('libs', nargs='*')
    ap.add_argument('--env', default='MO-Walker2d-v2')
    ap.add_argument('--tasks', type=int, default=40)
    ap.add_argument('--N', type=int, default=4)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--child', action='store_true')
    a = ap.parse_args()
    if a.child:
        return child(a)
    for lib in a.libs:
        env = dict(os.environ, PGM_LIB=lib)
        cmd = [sys.executable, __file__, '--child', '--env', a.env, '--tasks', str(a.tasks), '--N', str(a.N),
               '--reps', str(a.reps)]
        r = subprocess.run(cmd, env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == '__main__':
    main()
