"""Hypervolume at an equal env-step budget: device MOPG warm-up stage vs the fp64 CPU oracle.

The second half of BASELINE.json's metric ("hypervolume@budget").  Both sides run the PG-MORL warm-up
stage (morl/morl.py:50-99 with morl/warm_up.py:24-77): one task per weight of the warm-up grid
(generate_weights_batch_dfs, morl/utils.py:67-78), every task `iters` MOPG iterations (morl/mopg.py:60-182)
from the same fp32-rounded reference-order initial policies and with the reference's own RNG draws
(torch.manual_seed(j) -> T x normal([N, A]), E x randperm(T*N); morl/mopg.py:96).  The external
Pareto archive is built from every offspring (morl/ep.py:23-31) and its hypervolume taken against the
origin (morl/hypervolume.py / scripts/plot/ep_batch_visualize_2d.py:23-45).

    # CPU (this container or the box's host cores): the oracle side, written as a JSON fixture
    python scripts/hv_budget.py oracle --env MO-Hopper-v2 --delta 0.25 --N 1 --iters 10 --out profiles/x.json
    # GPU: the device side, compared with that fixture
    python scripts/hv_budget.py device --ref profiles/x.json --out profiles/y.json

The oracle is test infrastructure (oracle/__init__.py): this script is a measurement harness, not product
code.  fp32 (device) and fp64 (oracle) trajectories of a chaotic rollout drift apart over thousands of
steps, so the comparison is on the budget-level quantities: HV, EP size, per-task final objectives.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pgmorl_amd import envspec, pareto  # noqa: E402


def make_args(env, N, T, E, M, num_env_steps):
    spec = envspec.make_spec(env)
    gamma = 0.99 if 'Humanoid' in env else 0.995
    return argparse.Namespace(
        env_name=env, obj_num=spec['obj_num'], num_env_steps=num_env_steps, seed=0, num_steps=T, num_processes=N,
        ppo_epoch=E, num_mini_batch=M, clip_param=0.2, value_loss_coef=0.5, entropy_coef=0.0, lr=3e-4,
        max_grad_norm=0.5, gamma=gamma, gae_lambda=0.95, use_gae=True, use_proper_time_limits=True, ob_rms=True,
        obj_rms=True, raw=True, eval_num=1, use_linear_lr_decay=True, lr_decay_ratio=1.0, layernorm=False)


def init_state_dicts(spec, P, seed):
    """Reference-order initial policies (warm-up order under manual_seed(seed)), fp32-rounded values."""
    from oracle.policy import make_policy
    torch.manual_seed(seed)
    sds = []
    for _ in range(P):
        pol = make_policy(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
        sds.append({k: v.float().double().clone() for k, v in pol.state_dict().items()})
    return sds


def host_draws(T, N, A, E):
    def fn(j):
        torch.manual_seed(j)
        noise = torch.stack([torch.normal(torch.zeros(N, A, dtype=torch.float64), torch.ones(N, A, dtype=torch.float64))
                             for _ in range(T)])
        return noise.float().double(), [torch.randperm(T * N) for _ in range(E)]
    return fn


def _oracle_task(job):
    torch.set_num_threads(1)
    from oracle.mopg import initial_sample, mopg_worker
    cfg, p, sd, w = job
    args = make_args(cfg['env'], cfg['N'], cfg['T'], cfg['E'], cfg['M'], cfg['num_env_steps'])
    spec = envspec.make_spec(cfg['env'])
    sample = initial_sample(args, spec)
    sample.actor_critic.load_state_dict(sd)
    s0_train = envspec.reset_table(spec['obs_dim'], 0, cfg['N'])
    s0_eval = envspec.reset_table(spec['obs_dim'], 0, 1)
    fn = host_draws(cfg['T'], cfg['N'], spec['act_dim'], cfg['E'])
    offs = mopg_worker(args, spec, s0_train, s0_eval, sample, np.asarray(w), 0, cfg['iters'], noise_fn=fn)
    return p, [o.objs.tolist() for o in offs]


def summary(objs_per_task):
    flat = [o for task in objs_per_task for o in task]
    idx = pareto.get_ep_indices(np.asarray(flat))
    front = np.asarray(flat)[idx] if len(idx) else np.zeros((0, len(flat[0])))
    return {'hv': pareto.compute_hypervolume(front), 'ep_size': int(len(idx)), 'ep_indices': [int(i) for i in idx],
            'sparsity': pareto.compute_sparsity(front)}


def run_oracle(a):
    import multiprocessing as mp
    spec = envspec.make_spec(a.env)
    weights = pareto.weight_grid(spec['obj_num'], a.delta)
    P = len(weights)
    cfg = dict(env=a.env, N=a.N, T=a.T, E=a.E, M=a.M, iters=a.iters, num_env_steps=a.num_env_steps, seed=a.seed)
    sds = init_state_dicts(spec, P, a.seed)
    t0 = time.time()
    with mp.get_context('fork').Pool(min(a.procs, P)) as pool:
        res = dict(pool.map(_oracle_task, [(cfg, p, sds[p], list(weights[p])) for p in range(P)]))
    dt = time.time() - t0
    objs = [res[p] for p in range(P)]
    out = dict(cfg, side='oracle', tasks=P, weights=[list(map(float, w)) for w in weights],
               budget_env_steps=P * a.iters * a.T * a.N, objs=objs, wall_s=dt, procs=min(a.procs, P), **summary(objs))
    return out


def run_device(a):
    from pgmorl_amd.runtime import TaskBatch
    ref = json.load(open(a.ref))
    env, N, T, E, M, iters = ref['env'], ref['N'], ref['T'], ref['E'], ref['M'], ref['iters']
    spec = envspec.make_spec(env)
    weights = [np.asarray(w) for w in ref['weights']]
    P = len(weights)
    args = make_args(env, N, T, E, M, ref['num_env_steps'])
    tb = TaskBatch(env, P, num_processes=N, num_steps=T, ppo_epoch=E, num_mini_batch=M, gamma=args.gamma)
    tb.reset_stats()
    for p, sd in enumerate(init_state_dicts(spec, P, ref['seed'])):
        tb.set_task(p, sd, None, None, weights[p])
    tb.env_reset()
    total = int(ref['num_env_steps']) // T // N
    fn = host_draws(T, N, spec['act_dim'], E)
    objs = [[] for _ in range(P)]
    torch.cuda.synchronize()
    t0 = time.time()
    for j in range(iters):
        noise, perms = fn(j)
        lr = args.lr * (1.0 - j / float(total))
        tb.iteration(j, lr, noise=noise.float().to(tb.dev), perms=torch.stack(perms).numpy().astype(np.int32),
                     carry=j > 0)
        o = tb.objs.cpu().numpy()
        for p in range(P):
            objs[p].append(o[p].tolist())
    torch.cuda.synchronize()
    dt = time.time() - t0
    out = dict(env=env, N=N, T=T, E=E, M=M, iters=iters, num_env_steps=ref['num_env_steps'], seed=ref['seed'],
               side='device', tasks=P, budget_env_steps=P * iters * T * N, objs=objs, wall_s=dt, **summary(objs))
    hv_o, hv_d = ref['hv'], out['hv']
    fin_o = np.asarray([t[-1] for t in ref['objs']])
    fin_d = np.asarray([t[-1] for t in objs])
    out['vs_oracle'] = {
        'hv_oracle': hv_o, 'hv_device': hv_d, 'hv_rel_diff': (hv_d - hv_o) / max(abs(hv_o), 1e-12),
        'ep_size_oracle': ref['ep_size'], 'ep_size_device': out['ep_size'],
        'ep_indices_equal': ref['ep_indices'] == out['ep_indices'],
        'final_objs_max_rel_diff': float(np.max(np.abs(fin_d - fin_o) / np.maximum(np.abs(fin_o), 1e-9))),
        'oracle_wall_s': ref['wall_s'], 'oracle_procs': ref['procs']}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('side', choices=['oracle', 'device'])
    ap.add_argument('--env', default='MO-Hopper-v2')
    ap.add_argument('--delta', type=float, default=0.25, help='warm-up weight grid step (0.25 -> 5 tasks)')
    ap.add_argument('--N', type=int, default=1)
    ap.add_argument('--T', type=int, default=2048)
    ap.add_argument('--E', type=int, default=10)
    ap.add_argument('--M', type=int, default=32)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--num-env-steps', type=int, default=8_000_000)
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--procs', type=int, default=8)
    ap.add_argument('--ref', help='oracle JSON (device side)')
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    out = run_oracle(a) if a.side == 'oracle' else run_device(a)
    with open(a.out, 'w') as f:
        json.dump(out, f)
    brief = {k: out[k] for k in ('side', 'env', 'tasks', 'iters', 'budget_env_steps', 'hv', 'ep_size', 'wall_s')}
    if 'vs_oracle' in out:
        brief['vs_oracle'] = out['vs_oracle']
    print(json.dumps(brief))


if __name__ == '__main__':
    main()
