"""Warm-up policy initialisation (host, once per run) and the reference-compatible Policy module.

Initial parameters come from torch exactly as the reference draws them: under float64 default
dtype (morl/run.py:53), each ``nn.Linear`` default init followed by an orthogonal re-init
(gain sqrt(2) for the towers and value head, 1 for the action mean), including MLPBase's
discarded 1-output critic head, in module-construction order (a2c_ppo_acktr/model.py:201-256,
distributions.py:71-79, utils.py:53-57).  This is plumbing at the warm-up boundary; the hot path
never runs on the CPU.

``Policy`` is a torch module with the reference's state_dict keys so that ``final/EP_policy_i.pt``
files written by this build load into the reference's ``Policy`` and vice versa.
"""
import numpy as np
import torch
import torch.nn as nn


class _AddBias(nn.Module):
    def __init__(self, n):
        super().__init__()
        self._bias = nn.Parameter(torch.zeros(n).unsqueeze(1))

    def forward(self, x):
        return x + self._bias.t().view(1, -1)


class _Gaussian(nn.Module):
    def __init__(self, hidden, act_dim):
        super().__init__()
        self.fc_mean = nn.Linear(hidden, act_dim)
        nn.init.orthogonal_(self.fc_mean.weight.data, gain=1.0)
        nn.init.constant_(self.fc_mean.bias.data, 0.0)
        self.logstd = _AddBias(act_dim)


class _Base(nn.Module):
    def __init__(self, obs_dim, obj_num, hidden):
        super().__init__()
        gain = np.sqrt(2)

        def lin(i, o):
            m = nn.Linear(i, o)
            nn.init.orthogonal_(m.weight.data, gain=gain)
            nn.init.constant_(m.bias.data, 0.0)
            return m

        self.actor = nn.Sequential(lin(obs_dim, hidden), nn.Tanh(), lin(hidden, hidden), nn.Tanh())
        self.critic = nn.Sequential(lin(obs_dim, hidden), nn.Tanh(), lin(hidden, hidden), nn.Tanh())
        self.critic_linear = lin(hidden, 1)         # MLPBase head: drawn, then replaced
        self.critic_linear = lin(hidden, obj_num)   # MOMLPBase head


class Policy(nn.Module):
    """Parameter container with the reference's module tree / state_dict keys."""

    def __init__(self, obs_dim, act_dim, obj_num, hidden=64):
        super().__init__()
        self.base = _Base(obs_dim, obj_num, hidden)
        self.dist = _Gaussian(hidden, act_dim)


def new_policy(obs_dim, act_dim, obj_num, hidden=64):
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return Policy(obs_dim, act_dim, obj_num, hidden).double()
    finally:
        torch.set_default_dtype(prev)
