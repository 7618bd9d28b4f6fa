"""Oracle: actor-critic policy with a diagonal Gaussian head (torch CPU, fp64).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates:
  * Policy.act / get_value / evaluate_actions   -- a2c_ppo_acktr/model.py:57-82
  * MLPBase / MOMLPBase (two tanh MLPs, H=64)   -- a2c_ppo_acktr/model.py:201-256
  * DiagGaussian (+ FixedNormal patches)         -- a2c_ppo_acktr/distributions.py:29-40,71-90
  * AddBias, init                               -- a2c_ppo_acktr/utils.py:32-43,53-57

Modules are created in the reference's construction order so that the torch
RNG draws (nn.Linear default init, then orthogonal re-init, including the
discarded 1-output critic_linear of MLPBase) reproduce the reference's initial
parameters under the same ``torch.manual_seed``.  The state_dict keys equal the
reference's.
"""
import math

import numpy as np
import torch
import torch.nn as nn


def _orth(module, gain):
    nn.init.orthogonal_(module.weight.data, gain=gain)
    if module.bias is not None:
        nn.init.constant_(module.bias.data, 0)
    return module


class AddBias(nn.Module):
    def __init__(self, bias):
        super().__init__()
        self._bias = nn.Parameter(bias.unsqueeze(1))

    def forward(self, x):
        return x + self._bias.t().view(1, -1)


class DiagGaussian(nn.Module):
    def __init__(self, num_inputs, num_outputs):
        super().__init__()
        self.fc_mean = _orth(nn.Linear(num_inputs, num_outputs), 1.0)
        self.logstd = AddBias(torch.zeros(num_outputs))

    def forward(self, x):
        mean = self.fc_mean(x)
        logstd = self.logstd(torch.zeros(mean.size(), dtype=mean.dtype))
        return torch.distributions.Normal(mean, logstd.exp())


class MOMLPBase(nn.Module):
    def __init__(self, num_inputs, hidden_size=64, layernorm=False, obj_num=2):
        super().__init__()
        g = np.sqrt(2)

        def tower():
            mods, last = [], num_inputs
            for _ in range(2):
                mods.append(_orth(nn.Linear(last, hidden_size, bias=not layernorm), g))
                if layernorm:
                    mods.append(nn.LayerNorm(hidden_size, elementwise_affine=True))
                mods.append(nn.Tanh())
                last = hidden_size
            return nn.Sequential(*mods)

        self.actor = tower()
        self.critic = tower()
        # MLPBase builds a 1-output head first (consumes RNG), MOMLPBase replaces it.
        self.critic_linear = _orth(nn.Linear(hidden_size, 1), g)
        self.critic_linear = _orth(nn.Linear(hidden_size, obj_num), g)

    def forward(self, x):
        return self.critic_linear(self.critic(x)), self.actor(x)


class Policy(nn.Module):
    def __init__(self, obs_dim, act_dim, obj_num, hidden_size=64, layernorm=False):
        super().__init__()
        self.base = MOMLPBase(obs_dim, hidden_size, layernorm, obj_num)
        self.dist = DiagGaussian(hidden_size, act_dim)

    def _dist(self, x):
        value, feat = self.base(x)
        return value, self.dist(feat)

    def act(self, x, deterministic=False, noise=None):
        """Returns (value, action, action_log_probs).

        ``noise`` (same shape as the action) replaces the RNG draw of
        ``Normal.sample`` == torch.normal(mean, std) == z*std + mean.
        """
        value, dist = self._dist(x)
        if deterministic:
            action = dist.mean
        elif noise is not None:
            action = noise.to(dist.mean.dtype).mul(dist.scale).add(dist.mean)
        else:
            action = dist.sample()
        logp = dist.log_prob(action).sum(-1, keepdim=True)
        return value, action, logp

    def get_value(self, x):
        return self.base(x)[0]

    def evaluate_actions(self, x, action):
        value, dist = self._dist(x)
        logp = dist.log_prob(action).sum(-1, keepdim=True)
        entropy = dist.entropy().sum(-1).mean()
        return value, logp, entropy


def make_policy(obs_dim, act_dim, obj_num, hidden_size=64, layernorm=False):
    """Build a Policy under float64 default dtype (morl/run.py:53, warm_up.py:34-40)."""
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return Policy(obs_dim, act_dim, obj_num, hidden_size, layernorm).double()
    finally:
        torch.set_default_dtype(prev)


LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))
