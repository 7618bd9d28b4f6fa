"""Generation-boundary host logic: Pareto archive (EP), optimisation graph, weight grid,
hypervolume and sparsity.  Runs once per generation on the host.

Semantics follow the reference exactly (bit-exact EP membership and order):
  * get_ep_indices: indices ordered by np.argsort(obj0) (numpy default kind), keep points that are
    non-negative and not dominated (>= all, > any) by any point      -- morl/utils.py:24-39
  * EP.update: append every offspring, then keep EP indices           -- morl/ep.py:11-31
  * generate_weights_batch_dfs: accumulating w += delta (float quirks) -- morl/utils.py:67-78
  * OptGraph.insert                                                    -- morl/opt_graph.py:8-27
  * hypervolume w.r.t. the origin (maximisation), rounded to 4 dp      -- morl/hypervolume.py:41-74
  * sparsity                                                           -- morl/utils.py:87-100
The dominance test is an O(n log n) sort-and-sweep for two objectives (exact: the same boolean predicate)
and the native pairwise test (libpgm_host.so pgm_ep_mask) for more, instead of the reference's per-point
Python loop.
"""
import numpy as np

from . import _host


def _dominated_2d(objs):
    """Exact dominance flags of 2-D points in O(n log n): sorted by x descending (y descending inside equal x),
    point i is dominated iff some point with a strictly larger x has y >= y_i, or some point with an equal x
    has a strictly larger y (the same predicate as the pairwise >= all & > any test)."""
    x, y = objs[:, 0], objs[:, 1]
    order = np.lexsort((-y, -x))
    xs, ys = x[order], y[order]
    n = len(xs)
    start = np.ones(n, dtype=bool)
    start[1:] = xs[1:] != xs[:-1]
    gstart = np.maximum.accumulate(np.where(start, np.arange(n), 0))  # first index of each point's x group
    pm = np.maximum.accumulate(ys)
    before = np.where(gstart > 0, pm[np.maximum(gstart - 1, 0)], -np.inf)  # max y over strictly larger x
    dom_sorted = (before >= ys) | (ys[gstart] > ys)
    dom = np.empty(n, dtype=bool)
    dom[order] = dom_sorted
    return dom


def get_ep_indices(obj_batch_input):
    if len(obj_batch_input) == 0:
        return np.array([])
    objs = np.asarray(obj_batch_input, dtype=np.float64)
    if objs.shape[1] == 2 and not np.isnan(objs).any():
        keep = (objs >= 0).all(1) & ~_dominated_2d(objs)
    else:  # libpgm_host.so pgm_ep_mask: the reference's pairwise predicate in C++
        keep = _host.ep_mask(objs)
    order = np.argsort(objs.T[0])
    return [int(i) for i in order if keep[i]]


class EP:
    """External Pareto archive of Samples."""

    def __init__(self):
        self.obj_batch = np.array([])
        self.sample_batch = np.array([])

    def index(self, indices):
        idx = np.array(indices, dtype=int)
        self.obj_batch, self.sample_batch = self.obj_batch[idx], self.sample_batch[idx]

    def update(self, sample_batch):
        sample_batch = list(sample_batch)
        arr = np.empty(len(sample_batch), dtype=object)
        arr[:] = sample_batch
        self.sample_batch = np.append(self.sample_batch, arr)
        if sample_batch:  # the reference appends row by row (morl/ep.py:25-28); one vstack gives the same array
            new = np.array([s.objs for s in sample_batch])
            self.obj_batch = np.vstack([self.obj_batch, new]) if len(self.obj_batch) > 0 else new
        if len(self.obj_batch) == 0:
            return
        self.index(get_ep_indices(self.obj_batch))


class OptGraph:
    """Optimisation history: a rooted forest of (normalised weight, objs, parent) nodes."""

    def __init__(self):
        self.weights, self.objs, self.delta_objs, self.prev, self.succ = [], [], [], [], []

    def insert(self, weights, objs, prev):
        if hasattr(weights, 'detach'):  # a scalarisation's torch weight vector
            weights = weights.detach().cpu().numpy()
        w = np.array(weights, dtype=np.float64)
        self.weights.append(w / np.linalg.norm(w))
        objs = np.array(objs, dtype=np.float64)
        self.objs.append(objs)
        self.prev.append(prev)
        self.delta_objs.append(np.zeros_like(objs) if prev == -1 else objs - self.objs[prev])
        if prev != -1:
            self.succ[prev].append(len(self.objs) - 1)
        self.succ.append([])
        return len(self.objs) - 1


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


def weight_grid(obj_num, delta_weight, min_weight=0.0, max_weight=1.0):
    out = []
    generate_weights_batch_dfs(0, obj_num, min_weight, max_weight, delta_weight, [], out)
    return out


def _volume(points):
    """Dominated volume of the union of boxes [0, p], all p >= 0 (slicing along the last axis)."""
    if len(points) == 0:
        return 0.0
    if points.shape[1] == 1:
        return float(points[:, 0].max())
    if points.shape[1] == 2:  # sweep: sort by x descending, accumulate the staircase
        pts = points[np.argsort(-points[:, 0], kind='stable')]
        vol, ymax = 0.0, 0.0
        for i in range(len(pts)):
            x_next = pts[i + 1, 0] if i + 1 < len(pts) else 0.0
            ymax = max(ymax, pts[i, 1])
            vol += (pts[i, 0] - x_next) * ymax
        return vol
    pts = points[np.argsort(-points[:, -1], kind='stable')]
    vol = 0.0
    for i in range(len(pts)):
        lo = pts[i + 1, -1] if i + 1 < len(pts) else 0.0
        if pts[i, -1] > lo:
            vol += (pts[i, -1] - lo) * _volume(pts[:i + 1, :-1])
    return vol


def compute_hypervolume(front):
    f = np.array(front, dtype=np.float64)
    if f.size == 0:
        return 0.0
    f = f[(f >= 0).all(axis=1)]
    return round(_volume(f), 4)


def compute_sparsity(front):
    if len(front) < 2:
        return 0.0
    f = np.array(front, dtype=np.float64)
    s = sum(float(np.sum(np.square(np.diff(np.sort(f[:, d]))))) for d in range(f.shape[1]))
    return s / (len(front) - 1)
