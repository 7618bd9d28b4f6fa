"""Prototype measurement: the per-GPU population run as G independent task groups, each a TaskBatch on its own
stream (plus its own evaluation side stream), so the groups' iterations drift out of phase and their PPO updates
(which use 8 CUs per task at P <= 32) overlap other groups' rollouts instead of all tasks updating at once.

One step = one MOPG iteration of every task (as bench.py); value = tasks * N * T * steps / wall time.
Usage (GPU box): GPU_MAX_HW_QUEUES=8 python scripts/group_bench.py --groups 4 [--tasks 40 --steps 10 --warmup 3]
Measurement tool, not product code."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pgmorl_amd import envspec
from pgmorl_amd.policy import new_policy
from pgmorl_amd.runtime import TaskBatch

ap = argparse.ArgumentParser()
ap.add_argument('--env-name', default='MO-Walker2d-v2')
ap.add_argument('--tasks', type=int, default=40)
ap.add_argument('--groups', type=int, default=4)
ap.add_argument('--steps', type=int, default=10)
ap.add_argument('--warmup', type=int, default=3)
ap.add_argument('--num-processes', type=int, default=4)
ap.add_argument('--stagger-ms', type=float, default=0.0, help='group g starts g * this later (a spin kernel)')
args = ap.parse_args()

spec = envspec.make_spec(args.env_name)
N, T, P, G = args.num_processes, 2048, args.tasks, args.groups
sizes = [P // G + (1 if g < P % G else 0) for g in range(G)]
torch.manual_seed(0)
w = np.linspace(0, 1, P)
tbs, streams, k = [], [], 0
for g, pg in enumerate(sizes):
    tb = TaskBatch(args.env_name, pg, num_processes=N, num_steps=T, device='cuda')
    for p in range(pg):
        pol = new_policy(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
        tb.set_task(p, pol.state_dict(), {}, None, [w[k], 1 - w[k]])
        k += 1
    tb.env_reset()
    tbs.append(tb)
    streams.append(torch.cuda.Stream())
torch.cuda.synchronize()
total_updates = 5_000_000 // T // N


def step(j):
    for tb, s in zip(tbs, streams):
        with torch.cuda.stream(s):
            tb.iteration(j, 3e-4 * (1 - j / total_updates), carry=True, overlap_eval=True)


j = 0
for _ in range(args.warmup):
    step(j)
    j += 1
torch.cuda.synchronize()
t0 = time.perf_counter()
# phase offsets: group g's stream first spins g * stagger-ms (subtracted from the timed region below)
if args.stagger_ms > 0:
    for g, s in enumerate(streams):
        if g:
            with torch.cuda.stream(s):
                torch.cuda._sleep(int(g * args.stagger_ms * 1e-3 * 2.1e9))
for _ in range(args.steps):
    step(j)
    j += 1
torch.cuda.synchronize()
dt = time.perf_counter() - t0 - (G - 1) * args.stagger_ms * 1e-3
for tb in tbs:
    tb.check_update()
print(json.dumps({'groups': G, 'sizes': sizes, 'stagger_ms': args.stagger_ms, 'hw_queues': os.environ.get('GPU_MAX_HW_QUEUES'),
                  'ms_per_step': 1e3 * dt / args.steps, 'value': P * N * T * args.steps / dt}))
