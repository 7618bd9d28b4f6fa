"""Shared builders for the parity tests: matched oracle (fp64 CPU) and device (fp32 MI355X) states."""
import argparse

import numpy as np
import torch

from oracle.policy import make_policy
from pgmorl_amd import envspec


def small_args(env_name='MO-Hopper-v2', **kw):
    spec = envspec.make_spec(env_name)
    a = dict(env_name=env_name, obj_num=spec['obj_num'], num_env_steps=10 ** 9, seed=0, num_steps=64,
             num_processes=4, ppo_epoch=2, num_mini_batch=4, clip_param=0.2, value_loss_coef=0.5,
             entropy_coef=0.0, lr=3e-4, max_grad_norm=0.5, gamma=0.995, gae_lambda=0.95, use_gae=True,
             use_proper_time_limits=True, ob_rms=True, obj_rms=True, raw=True, eval_num=1,
             use_linear_lr_decay=True, lr_decay_ratio=1.0, layernorm=False)
    a.update(kw)
    return argparse.Namespace(**a)


def fp32_policies(spec, P, seed=0):
    """P reference-initialised policies (warm-up order under manual_seed(seed)) with parameters
    rounded to fp32 so the oracle and the device start from identical values."""
    torch.manual_seed(seed)
    pols = []
    for _ in range(P):
        pol = make_policy(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
        with torch.no_grad():
            for prm in pol.parameters():
                prm.copy_(prm.float().double())
        pols.append(pol)
    return pols


def perturb(pol, scale, gen):
    """Break the zero-bias / zero-logstd symmetry so every code path sees non-trivial values."""
    with torch.no_grad():
        for prm in pol.parameters():
            prm.add_((torch.randn(prm.shape, generator=gen, dtype=torch.float64) * scale).float().double())
    return pol


def weights_grid(K, P):
    rng = np.random.RandomState(7)
    w = rng.dirichlet(np.ones(K), size=P)
    return w
