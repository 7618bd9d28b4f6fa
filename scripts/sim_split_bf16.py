"""Precision study (CPU, exploratory): would the PPO update's matrix products on the bf16 matrix cores with split
operands keep the fp32 parity tests' tolerance?  x = hi + lo (+ lo2) with bf16 planes; a product of two split values
as the sum of the plane products that matter (2 planes: hi.hi + hi.lo + lo.hi, ~2^-16 relative; 3 planes: six
products, ~2^-24).  Every nn.Linear of the oracle policy (forward, input gradient, weight gradient) runs its products
through the emulation (bf16 plane products are exact in fp32, accumulated in fp32); everything else is fp32.

Arms, from the same fp32-rounded parameters and inputs, one task's full update (E epochs x M minibatches):
  fp64 (the oracle, the truth), fp32 (exact fp32 products: the f32 MFMA kernels), bf16x3 (2 planes), bf16x6 (3 planes).
Reported: the max of |p - p64| / (2e-6 + 1e-5 |p64|) over every parameter (the parity tests' criterion, <= 1 passes)
and the max |dp|.  Test infrastructure: runs the oracle.

    python scripts/sim_split_bf16.py [--epochs 10] [--T 2048]
"""
import argparse
import copy
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as Fn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ppo as oppo  # noqa: E402
from oracle.policy import make_policy  # noqa: E402
from pgmorl_amd import envspec  # noqa: E402

MODE = {'planes': 0}


def split(x, n):
    """n bf16 planes of fp32 x (round to nearest even), as fp32 tensors."""
    out, r = [], x
    for _ in range(n):
        h = r.to(torch.bfloat16).to(torch.float32)
        out.append(h)
        r = r - h
    return out


def mm(a, b):
    n = MODE['planes']
    if n == 0:
        return a @ b
    A, B = split(a, n), split(b, n)
    if n == 2:
        terms = [(0, 0), (0, 1), (1, 0)]
    else:
        terms = [(0, 0), (0, 1), (1, 0), (0, 2), (1, 1), (2, 0)]
    acc = torch.zeros(a.shape[0], b.shape[1], dtype=torch.float32)
    for i, j in reversed(terms):  # small terms first
        acc = acc + A[i] @ B[j]
    return acc


class Lin(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        y = mm(x, w.t())
        return y + b if b is not None else y

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        return mm(g, w), mm(g.t(), x), g.sum(0)


def patched_linear(x, w, b=None):
    if x.dtype == torch.float32 and MODE['planes']:
        return Lin.apply(x, w, b)
    return ORIG(x, w, b)


ORIG = Fn.linear


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--env', default='MO-Walker2d-v2')
    ap.add_argument('--T', type=int, default=2048)
    ap.add_argument('--N', type=int, default=4)
    ap.add_argument('--epochs', type=int, default=10)
    ap.add_argument('--M', type=int, default=32)
    ap.add_argument('--seeds', type=int, nargs='+', default=[0, 1])
    a = ap.parse_args()
    nn.functional.linear = patched_linear
    spec = envspec.make_spec(a.env)
    O, A, K = spec['obs_dim'], spec['act_dim'], spec['obj_num']
    T, N, E, M = a.T, a.N, a.epochs, a.M
    B = T * N
    for seed in a.seeds:
        torch.manual_seed(seed)
        base = make_policy(O, A, K)
        with torch.no_grad():
            for p in base.parameters():
                p.add_(torch.randn_like(p) * 0.05)
                p.copy_(p.float().double())
        rng = np.random.RandomState(seed)
        obs = torch.from_numpy(np.clip(rng.randn(T + 1, N, O), -3, 3).astype(np.float32)).double()
        with torch.no_grad():
            v, act, lp = base.act(obs[:T].reshape(B, O), noise=torch.from_numpy(rng.randn(B, A)))
        act = act.float().double().reshape(T, N, A)
        lp = (lp[:, 0] + torch.from_numpy(rng.randn(B) * 0.05)).float().double().reshape(T, N, 1)
        vals = torch.cat([(v + torch.from_numpy(rng.randn(B, K) * 0.1)).float().double().reshape(T, N, K),
                          torch.zeros(1, N, K, dtype=torch.float64)])
        rets = (vals + torch.from_numpy(rng.randn(T + 1, N, K) * 0.5)).float().double()
        adv = torch.from_numpy(rng.randn(T, N, 1)).float().double()
        perms = [torch.randperm(B, generator=torch.Generator().manual_seed(seed * 10 + e)) for e in range(E)]
        res = {}
        for arm, planes in (('fp64', None), ('fp32', 0), ('bf16x3', 2), ('bf16x6', 3)):
            pol = copy.deepcopy(base)
            if planes is not None:
                pol = pol.float()
            MODE['planes'] = planes or 0
            agent = oppo.PPO(pol, 0.2, E, M, 0.5, 0.0, lr=3e-4, eps=1e-5, max_grad_norm=0.5)
            ro = oppo.RolloutStorage(T, N, O, A, K)
            ro.obs.copy_(obs)
            ro.actions.copy_(act)
            ro.action_log_probs.copy_(lp)
            ro.value_preds.copy_(vals)
            ro.returns.copy_(rets)
            for e in range(E):
                for mbt in ro.minibatches(adv[..., 0], M, perms[e]):
                    agent.minibatch_step(*mbt)
            res[arm] = torch.cat([p.detach().double().flatten() for p in pol.parameters()])
        ref = res['fp64']
        line = [f'seed {seed}']
        for arm in ('fp32', 'bf16x3', 'bf16x6'):
            d = (res[arm] - ref).abs()
            line.append(f'{arm}: crit {float((d / (2e-6 + 1e-5 * ref.abs())).max()):.3f} max|dp| {float(d.max()):.2e}')
        print(' | '.join(line), flush=True)


if __name__ == '__main__':
    main()
