"""Oracle: Pareto archive, hypervolume, sparsity, weight grid, optimisation graph (numpy, fp64).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates:
  * check_dominated / get_ep_indices (argsort on obj0, non-negative, not dominated)
                                                    -- morl/utils.py:24-39
  * EP.update (append all, keep EP indices)         -- morl/ep.py:11-31
  * generate_weights_batch_dfs (accumulating w += delta, float quirks kept)
                                                    -- morl/utils.py:67-78
  * compute_sparsity                                -- morl/utils.py:87-100
  * OptGraph.insert                                 -- morl/opt_graph.py:8-27
  * hypervolume w.r.t. the origin, maximisation, rounded to 4 dp
    (morl/hypervolume.py:41-74 computes it with the Fonseca dimension sweep; this
    restatement uses exact inclusion by recursive slicing and the 2-D sweep of
    scripts/plot/ep_batch_visualize_2d.py:23-45)
"""
import numpy as np


def check_dominated(obj_batch, obj):
    return np.logical_and((obj_batch >= obj).all(axis=1), (obj_batch > obj).any(axis=1)).any()


def get_ep_indices(obj_batch_input):
    if len(obj_batch_input) == 0:
        return np.array([])
    obj_batch = np.array(obj_batch_input)
    out = []
    for idx in np.argsort(obj_batch.T[0]):
        if (obj_batch[idx] >= 0).all() and not check_dominated(obj_batch, obj_batch[idx]):
            out.append(idx)
    return out


class EP:
    def __init__(self):
        self.obj_batch = np.array([])
        self.sample_batch = np.array([])

    def update(self, samples):
        self.sample_batch = np.append(self.sample_batch, np.array(list(samples), dtype=object))
        for s in samples:
            self.obj_batch = np.vstack([self.obj_batch, s.objs]) if len(self.obj_batch) > 0 else np.array([s.objs])
        if len(self.obj_batch) == 0:
            return
        keep = np.array(get_ep_indices(self.obj_batch), dtype=int)
        self.obj_batch, self.sample_batch = self.obj_batch[keep], self.sample_batch[keep]


def generate_weights_batch_dfs(i, obj_num, min_weight, max_weight, delta_weight, weight, weights_batch):
    if i == obj_num - 1:
        weight.append(1.0 - np.sum(weight[0:i]))
        weights_batch.append(list(weight))
        return
    w = min_weight
    while w < max_weight + 0.5 * delta_weight and np.sum(weight[0:i]) + w < 1.0 + 0.5 * delta_weight:
        weight.append(w)
        generate_weights_batch_dfs(i + 1, obj_num, min_weight, max_weight, delta_weight, weight, weights_batch)
        weight = weight[0:i]
        w += delta_weight


def compute_sparsity(front):
    if len(front) < 2:
        return 0.0
    f = np.array(front)
    s = 0.0
    for d in range(f.shape[1]):
        col = np.sort(f[:, d])
        s += np.sum(np.square(np.diff(col)))
    return s / (len(front) - 1)


def _hv_max(points):
    """Exact dominated volume of the union of boxes [0, p] (all p >= 0)."""
    if len(points) == 0:
        return 0.0
    m = points.shape[1]
    if m == 1:
        return float(points[:, 0].max())
    order = np.argsort(-points[:, -1], kind='stable')
    pts = points[order]
    vol = 0.0
    for i in range(len(pts)):
        hi = pts[i, -1]
        lo = pts[i + 1, -1] if i + 1 < len(pts) else 0.0
        if hi > lo:
            vol += (hi - lo) * _hv_max(pts[:i + 1, :-1])
    return vol


def compute_hypervolume(front):
    f = np.array(front, dtype=np.float64)
    if f.size == 0:
        return 0.0
    f = f[(f >= 0).all(axis=1)]
    return round(_hv_max(f), 4)


def hv_sparsity_2d(obj_batch, ref=(0.0, 0.0)):
    """scripts/plot/ep_batch_visualize_2d.py:10-45 (reported-metric form)."""
    obj_batch = np.array(obj_batch)
    order = np.lexsort((obj_batch.T[1], obj_batch.T[0]))
    idx, best = [], -np.inf
    for i in order[::-1]:
        if obj_batch[i][1] > best:
            best = obj_batch[i][1]
            idx.append(i)
    objs = obj_batch[idx[::-1]]
    x, hv, sp = ref[0], 0.0, 0.0
    for i in range(len(objs)):
        hv += (max(ref[0], objs[i][0]) - x) * (max(ref[1], objs[i][1]) - ref[1])
        x = max(ref[0], objs[i][0])
        if i > 0:
            sp += np.sum(np.square(objs[i] - objs[i - 1]))
    sp = 0.0 if len(objs) == 1 else sp / (len(objs) - 1)
    return hv, sp


class OptGraph:
    def __init__(self):
        self.weights, self.objs, self.delta_objs, self.prev, self.succ = [], [], [], [], []

    def insert(self, weights, objs, prev):
        w = np.array(weights, dtype=np.float64)
        self.weights.append(w / np.linalg.norm(w))
        self.objs.append(np.array(objs, copy=True))
        self.prev.append(prev)
        self.delta_objs.append(np.zeros_like(objs) if prev == -1 else objs - self.objs[prev])
        if prev != -1:
            self.succ[prev].append(len(self.objs) - 1)
        self.succ.append([])
        return len(self.objs) - 1
