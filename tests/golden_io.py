"""Readers for the committed golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load(name):
    with np.load(os.path.join(GOLDEN, name + '.npz')) as z:  # allow_pickle=False (numpy default)
        return {k: z[k] for k in z.files}


def state_dict(g, prefix):
    """Reference state_dict (fp64 torch tensors) stored under '<prefix>/<key>'."""
    n = len(prefix) + 1
    return {k[n:]: torch.from_numpy(np.array(v)) for k, v in g.items() if k.startswith(prefix + '/')}


class RMS:
    """Plain (mean, var, count) holder with the RunningMeanStd attribute names."""

    def __init__(self, mean, var, count):
        self.mean, self.var, self.count = mean, var, float(count)
