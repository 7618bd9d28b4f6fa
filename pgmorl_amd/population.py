"""Performance-buffer population and prediction-guided task selection (host, once per generation).

Drop-in for the reference's ``Population`` classes, selected by objective count like morl/morl.py:46-51:
  * Population2d -- morl/population_2d.py:123-319 (angular performance buffers, ±pi/4 weight fan,
    staircase hypervolume / EP-order sparsity of population_2d.py:185-202)
  * Population3d -- morl/population_3d.py:120-345 (buffer directions from the weight grid, random
    weight candidates within pi/4 of the last weight, InnerHyperVolume / utils.compute_sparsity)
  * predict_hyperbolic -- population_2d.py:27-118 / population_3d.py:23-112: per objective, a
    soft-L1 ``least_squares`` fit of f(x) = A (e^{a(x-b)} - 1) / (e^{a(x-b)} + 1) + c to the
    improvement deltas of nearby OptGraph nodes, Gaussian-weighted by objective distance.

Semantics kept: candidate construction and order, duplicate-direction filters, the greedy
argmax of HV - alpha * sparsity with first-max tie breaking, virtual-EP updates, the global
``np.random`` draws of ``random_selection`` and of the 3-D candidate shuffle.

Generation-boundary speed, results unchanged:
  * the hyperbolic fits of all population members run over a spawn pool of CPU-only workers
    (PGM_FIT_WORKERS, default min(15, CPUs - 1)), each the same least_squares call;
  * 2-D greedy steps screen every candidate with one vectorised pass and re-score exactly (the
    reference's own computation, strict > in index order) only those within a rounding bound of the
    best, so the pick and its tie-breaking are the reference's;
  * 3-D greedy steps score candidate chunks on the same pool (the reference forks one process per
    candidate, population_3d.py:216-237).

Deliberate differences (documented in DESIGN.md):
  * The 3-D candidate evaluation uses vectorised numpy (update_ep, prefix-area hypervolume); the
    order of float summation inside the hypervolume differs from InnerHyperVolume's (it is rounded
    to 4 dp like hypervolume.py:74).
  * The 2-D neighbourhood search (population_2d.py:37-54) has no exit when fewer than four
    distinct weights are reachable and spins forever; here it stops once a larger threshold
    cannot add any node.  When no node is reachable at all (the reference raises inside
    ``np.max`` of an empty array), the prediction is the unchanged objective vector.
  * scipy is the container's (1.15) rather than the pinned 1.4.1 (environment.yml:103): the
    fitted parameters are parity-unpinned beyond the tests' synthetic recoveries.
"""
from copy import deepcopy

import numpy as np
from scipy.optimize import least_squares

from .pareto import compute_sparsity as _sparsity_sorted
from .pareto import get_ep_indices, weight_grid

# --------------------------------------------------------------------------- prediction model


def collect_nearest_data(opt_graph, optgraph_id, threshold=0.1, objs_arr=None):
    """population_2d.py:11-21: (objs, sum-normalised next weight, delta objs) of every successor
    edge leaving a node within ``threshold`` (relative, per objective) of node ``optgraph_id``.
    ``objs_arr`` = np.array(opt_graph.objs), when the caller already holds it."""
    objs_data, weights_data, delta_objs_data = [], [], []
    objs_arr = np.asarray(opt_graph.objs, dtype=np.float64) if objs_arr is None else objs_arr
    center = objs_arr[optgraph_id]
    near = np.all(np.abs(center - objs_arr) < np.abs(center) * threshold, axis=1)
    for i in np.nonzero(near)[0]:
        for nxt in opt_graph.succ[i]:
            objs_data.append(opt_graph.objs[i])
            weights_data.append(opt_graph.weights[nxt] / np.sum(opt_graph.weights[nxt]))
            delta_objs_data.append(opt_graph.delta_objs[nxt])
    return objs_data, weights_data, delta_objs_data


def _count_distinct(weights_data, enough=4):
    cnt = 0
    for i in range(len(weights_data)):
        if all(np.linalg.norm(weights_data[i] - weights_data[j]) >= 1e-5 for j in range(i)):
            cnt += 1
            if cnt >= enough:
                break
    return cnt


def _max_useful_threshold(opt_graph, optgraph_id, objs_arr):
    """Smallest threshold beyond which collect_nearest_data cannot grow any more (nodes relative to a
    centre with a zero coordinate need diff < 0 there: never reachable)."""
    center = np.abs(objs_arr[optgraph_id])
    if np.any(center == 0):
        return 0.0
    has_succ = np.array([len(s) > 0 for s in opt_graph.succ])
    if not has_succ.any():
        return 0.0
    diff = np.abs(objs_arr[optgraph_id] - objs_arr[has_succ])
    return float(np.max(diff / center))


def _hyperbolic(x, A, a, b, c):
    e = np.exp(a * (x - b))
    return A * (e - 1) / (e + 1) + c


def predict_hyperbolic(args, opt_graph, optgraph_id, test_weights, bounded_search=False, objs_arr=None):
    """population_2d.py:27-118 (bounded_search=False) / population_3d.py:23-112 (True, which adds
    the ``threshold >= 1.0`` exit of population_3d.py:46)."""
    test_weights = np.array(test_weights, dtype=np.float64)
    test_weights = test_weights / test_weights.sum(axis=1, keepdims=True)
    objs_arr = np.asarray(opt_graph.objs, dtype=np.float64) if objs_arr is None else objs_arr
    threshold, sigma = 0.1, 0.03
    t_max = None if bounded_search else _max_useful_threshold(opt_graph, optgraph_id, objs_arr)
    while True:
        objs_data, weights_data, delta_objs_data = collect_nearest_data(opt_graph, optgraph_id, threshold, objs_arr)
        if _count_distinct(weights_data) > 3:
            break
        if bounded_search and threshold >= 1.0:
            break
        if not bounded_search and threshold > t_max:
            break
        threshold *= 2.0
        sigma *= 2.0

    original = np.asarray(opt_graph.objs[optgraph_id], dtype=np.float64)
    if len(objs_data) == 0:
        return {'sample_index': optgraph_id, 'predictions': [original.copy() for _ in range(len(test_weights))]}

    objs_data = np.array(objs_data, dtype=np.float64)
    weights_data = np.array(weights_data, dtype=np.float64)
    delta_objs_data = np.array(delta_objs_data, dtype=np.float64)
    dist = np.linalg.norm(np.abs(objs_data - original) / np.abs(original), axis=1)
    w = np.exp(-((dist / sigma) ** 2) / 2.0)

    def fun(p, x, y):
        return (_hyperbolic(x, *p) - y) * w

    def jac(p, x, y):
        A, a, b, _ = p
        e = np.exp(a * (x - b))
        J = np.empty((4, len(x)))
        J[0] = (e - 1) / (e + 1) * w
        J[1] = A * (x - b) * (2. * e) / ((e + 1) ** 2) * w
        J[2] = A * (-a) * (2. * e) / ((e + 1) ** 2) * w
        J[3] = w
        return J.T

    deltas = []
    for dim in range(args.obj_num):
        x, y = weights_data[:, dim], delta_objs_data[:, dim]
        a_hi = np.clip(np.max(y) - np.min(y), 1.0, 500.0)
        res = least_squares(fun, np.ones(4), loss='soft_l1', f_scale=20., args=(x, y), jac=jac,
                            bounds=([0, 0.1, -5., -500.], [a_hi, 20., 5., 500.]))
        deltas.append(_hyperbolic(test_weights.T[dim], *res.x))
    deltas = np.array(deltas).T
    return {'sample_index': optgraph_id, 'predictions': [original + deltas[i] for i in range(len(test_weights))]}


def _predict_chunk(payload):
    """Pool worker: predict_hyperbolic for a chunk of (node, test weights) jobs on a snapshot of the graph."""
    args_d, graph, jobs, bounded = payload
    import argparse
    args = argparse.Namespace(**args_d)
    og = _GraphView(*graph)
    objs_arr = np.asarray(og.objs, dtype=np.float64)
    return [predict_hyperbolic(args, og, node, tw, bounded_search=bounded, objs_arr=objs_arr) for node, tw in jobs]


class _GraphView:
    """The fields of an OptGraph that predict_hyperbolic reads (picklable snapshot for the fit workers)."""

    def __init__(self, weights, objs, delta_objs, succ):
        self.weights, self.objs, self.delta_objs, self.succ = weights, objs, delta_objs, succ


_POOL = None


def _fit_pool():
    """Lazily started spawn pool for the hyperbolic fits (CPU-only workers: numpy / scipy, no GPU runtime).
    Size: PGM_FIT_WORKERS, default min(15, usable CPUs - 1); 0 or 1 disables it."""
    global _POOL
    import os
    n = int(os.environ.get('PGM_FIT_WORKERS', min(15, max(1, len(os.sched_getaffinity(0)) - 1))))
    if n <= 1:
        return None
    if _POOL is None:
        import multiprocessing as mp
        import sys
        import types
        # workers start from a bare __main__ (not the caller's script, which may import torch and open the
        # GPU) with no device visible: CPU-only processes
        saved_main = sys.modules['__main__']
        saved_env = {k: os.environ.get(k) for k in ('HIP_VISIBLE_DEVICES', 'ROCR_VISIBLE_DEVICES')}
        sys.modules['__main__'] = types.ModuleType('__main__')
        os.environ['HIP_VISIBLE_DEVICES'] = os.environ['ROCR_VISIBLE_DEVICES'] = ''
        try:
            _POOL = mp.get_context('spawn').Pool(n)
        finally:
            sys.modules['__main__'] = saved_main
            for k, v in saved_env.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    return _POOL


def predict_all(args, opt_graph, jobs, bounded_search, min_parallel=16):
    """predict_hyperbolic for every (node, test_weights) job, in order: in-process for few jobs, else chunked
    over the fit pool (each chunk carries one snapshot of the graph)."""
    pool = _fit_pool() if len(jobs) >= min_parallel else None
    if pool is None:
        objs_arr = np.asarray(opt_graph.objs, dtype=np.float64)
        return [predict_hyperbolic(args, opt_graph, node, tw, bounded_search=bounded_search, objs_arr=objs_arr)
                for node, tw in jobs]
    graph = (list(opt_graph.weights), list(opt_graph.objs), list(opt_graph.delta_objs), [list(x) for x in opt_graph.succ])
    args_d = {'obj_num': args.obj_num}
    nch = min(len(jobs), 4 * pool._processes)
    chunks = [jobs[i::nch] for i in range(nch)]  # strided chunks balance cheap and expensive fits
    outs = pool.map(_predict_chunk, [(args_d, graph, ch, bounded_search) for ch in chunks])
    res = [None] * len(jobs)
    for i, out in enumerate(outs):
        res[i::nch] = out
    return res


def _screen_2d(ep, preds, alpha):
    """Vectorised HV - alpha * sparsity of (virtual EP + candidate) for every candidate (2 objectives), in a
    float order of its own (screening only: see Population2d._best_candidate).  Returns (scores, magnitude
    of the summed terms) for the rounding bound."""
    C, n = len(preds), len(ep)
    x0, x1 = preds[:, 0], preds[:, 1]
    if n:
        q0, q1 = ep[:, 0], ep[:, 1]
        dom_by_x = (x0[:, None] >= q0[None]) & (x1[:, None] >= q1[None]) & \
                   ((x0[:, None] > q0[None]) | (x1[:, None] > q1[None]))       # [C, n] EP point dropped
        x_dom = ((q0[None] >= x0[:, None]) & (q1[None] >= x1[:, None]) &
                 ((q0[None] > x0[:, None]) | (q1[None] > x1[:, None]))).any(1)  # candidate dropped
    else:
        dom_by_x = np.zeros((C, 0), dtype=bool)
        x_dom = np.zeros(C, dtype=bool)
    x_keep = ~x_dom & (x0 >= 0) & (x1 >= 0)
    # merged sequence per candidate: EP points (already obj0-ascending) with the candidate at its slot
    pos = np.searchsorted(ep[:, 0], x0, side='left') if n else np.zeros(C, dtype=int)
    j = np.arange(n + 1)[None, :]
    src = np.where(j < pos[:, None], j, j - 1)
    is_x = j == pos[:, None]
    src_c = np.clip(src, 0, max(n - 1, 0))
    p0 = np.where(is_x, x0[:, None], ep[src_c, 0] if n else 0.0)
    p1 = np.where(is_x, x1[:, None], ep[src_c, 1] if n else 0.0)
    keep = np.where(is_x, x_keep[:, None], ~np.take_along_axis(np.pad(dom_by_x, ((0, 0), (0, 1))), src_c, 1)
                    if n else False)
    # staircase HV: (x_i - x_prev) * y_i over kept points, x_prev the previous kept x (ascending)
    kx = np.where(keep, np.maximum(p0, 0.0), 0.0)
    prev = np.concatenate([np.zeros((C, 1)), np.maximum.accumulate(kx, axis=1)[:, :-1]], 1)
    terms = np.where(keep, (kx - prev) * np.maximum(p1, 0.0), 0.0)
    hv = terms.sum(1)
    # EP-order sparsity: squared steps between consecutive kept points
    big = np.where(keep, p0, np.nan)
    last0 = _ffill(big)
    last1 = _ffill(np.where(keep, p1, np.nan))
    d0 = p0 - np.concatenate([np.full((C, 1), np.nan), last0[:, :-1]], 1)
    d1 = p1 - np.concatenate([np.full((C, 1), np.nan), last1[:, :-1]], 1)
    step = np.where(keep & ~np.isnan(d0), d0 * d0 + d1 * d1, 0.0)
    cnt = keep.sum(1)
    sp = np.where(cnt >= 2, step.sum(1) / np.maximum(cnt - 1, 1), 0.0)
    mag = np.abs(terms).sum(1) + alpha * np.abs(step).sum(1) / np.maximum(cnt - 1, 1)
    return hv - alpha * sp, mag


def _ffill(a):
    """Forward-fill NaNs along axis 1."""
    idx = np.where(~np.isnan(a), np.arange(a.shape[1])[None, :], 0)
    np.maximum.accumulate(idx, axis=1, out=idx)
    out = np.take_along_axis(a, idx, 1)
    return out


# --------------------------------------------------------------------------- virtual EP metrics


def update_ep(ep_objs_batch, new_objs):
    """morl/utils.py:41-66, vectorised: drop EP points weakly dominated by ``new_objs``; insert it
    (before the first point with a larger obj0) unless an EP point beats it by more than 1e-5."""
    new_objs = np.asarray(new_objs, dtype=np.float64)
    ep = np.asarray(ep_objs_batch, dtype=np.float64).reshape(-1, len(new_objs))
    if (new_objs < 0).any():
        return ep.copy()
    keep = ~(new_objs >= ep).all(axis=1)
    beaten = ((ep >= new_objs - 1e-5).all(axis=1) & (ep > new_objs + 1e-5).any(axis=1)).any()
    out = ep[keep]
    if beaten:
        return out
    larger = np.nonzero(new_objs[0] < out[:, 0])[0]
    pos = int(larger[0]) if len(larger) else len(out)
    return np.insert(out, pos, new_objs, axis=0)


def hypervolume_nd(front):
    """Dominated volume w.r.t. the origin, rounded to 4 dp (morl/hypervolume.py:41-74 semantics:
    points with a negative coordinate do not count).  Slices along the last objective; each slice's
    area is computed for all prefixes at once as a masked running maximum over a global ordering."""
    f = np.asarray(front, dtype=np.float64)
    if f.size == 0:
        return 0.0
    f = f[(f >= 0).all(axis=1)]
    if len(f) == 0:
        return 0.0
    if f.shape[1] == 1:
        return round(float(f[:, 0].max()), 4)
    if f.shape[1] == 2:
        return round(_area_prefixes(f[:, :1], f[:, 1:2].T, np.ones((1, len(f)), bool))[0], 4)
    if f.shape[1] != 3:
        from .pareto import compute_hypervolume
        return compute_hypervolume(f)
    order = np.argsort(-f[:, 2], kind='stable')
    f = f[order]
    n = len(f)
    inc = np.tri(n, dtype=bool)                        # prefix i holds points 0..i (z descending)
    areas = _area_prefixes(f[:, :1], np.broadcast_to(f[:, 1], (n, n)), inc)
    z = f[:, 2]
    dz = z - np.append(z[1:], 0.0)
    return round(float(np.dot(areas, dz)), 4)


def _area_prefixes(x, y, inc):
    """Area of the union of boxes [0, x_j] x [0, y_j] over each row's included points."""
    xs = x[:, 0]
    o = np.argsort(-xs, kind='stable')
    dx = xs[o] - np.append(xs[o][1:], 0.0)
    h = np.where(inc[:, o], y[:, o], 0.0)
    return (np.maximum.accumulate(h, axis=1) * dx).sum(axis=1)


def _hv_2d_staircase(ep_objs):
    """population_2d.py:185-192: staircase over the EP (ascending obj0), reference point (0, 0)."""
    hv, x = 0.0, 0.0
    for o in ep_objs:
        hv += (max(0.0, o[0]) - x) * (max(0.0, o[1]) - 0.0)
        x = max(0.0, o[0])
    return hv


def _sparsity_ep_order(ep_objs):
    """population_2d.py:194-202: mean squared step between consecutive EP points."""
    if len(ep_objs) < 2:
        return 0.0
    return float(np.sum(np.square(np.diff(ep_objs, axis=0)))) / (len(ep_objs) - 1)


def _evaluate_3d(virtual_ep, pred):
    """population_3d.py:216-237 per candidate: update_ep, then hypervolume and sparsity of the new front."""
    e = update_ep(virtual_ep, pred)
    if len(e) == 0:
        return 0.0, 0.0
    return hypervolume_nd(e), _sparsity_sorted(e)


def _score_chunk_3d(payload):
    virtual_ep, preds = payload
    return np.array([_evaluate_3d(virtual_ep, x) for x in preds], dtype=np.float64).reshape(-1, 2)


# --------------------------------------------------------------------------- populations


class _PopulationBase:
    bounded_search = False

    def __init__(self, args):
        self.sample_batch = []
        self.pbuffer_size = args.pbuffer_size
        self.obj_num = args.obj_num
        self.z_min = np.zeros(args.obj_num)
        self.pbuffers = [[] for _ in range(self.pbuffer_num)]
        self.pbuffer_dist = [[] for _ in range(self.pbuffer_num)]

    def _insert_sorted(self, buffer_id, index, dist, enforce=False):
        buf, bd = self.pbuffers[buffer_id], self.pbuffer_dist[buffer_id]
        inserted = False
        for i in range(len(buf)):
            if bd[i] < dist:
                buf.insert(i, index)
                bd.insert(i, dist)
                inserted = True
                break
        if enforce:
            if not inserted:
                buf.append(index)
                bd.append(dist)
            return True
        if inserted and len(buf) > self.pbuffer_size:
            del buf[self.pbuffer_size:]
            del bd[self.pbuffer_size:]
        elif not inserted and len(buf) < self.pbuffer_size:
            buf.append(index)
            bd.append(dist)
            inserted = True
        return inserted

    def update(self, sample_batch):
        """Union of population and offspring, re-bucketed (population_2d.py:169-183)."""
        all_sample_batch = list(self.sample_batch) + list(sample_batch)
        self.sample_batch = []
        self.pbuffers = [[] for _ in range(self.pbuffer_num)]
        self.pbuffer_dist = [[] for _ in range(self.pbuffer_num)]
        for i, s in enumerate(all_sample_batch):
            self.insert_pbuffer(i, s.objs)
        for buf in self.pbuffers:
            for idx in buf:
                self.sample_batch.append(all_sample_batch[idx])

    def random_selection(self, args, scalarization_template):
        """population_2d.py:308-319 (global np.random stream)."""
        elite_batch, scalarization_batch = [], []
        for _ in range(args.num_tasks):
            elite_batch.append(self.sample_batch[np.random.choice(len(self.sample_batch))])
            w = np.random.uniform(args.min_weight, args.max_weight, args.obj_num)
            sc = deepcopy(scalarization_template)
            sc.update_weights(w / np.sum(w))
            scalarization_batch.append(sc)
        return elite_batch, scalarization_batch

    # the greedy knapsack over predicted offspring (population_2d.py:262-304, population_3d.py:296-333)
    def prediction_guided_selection(self, args, iteration, ep, opt_graph, scalarization_template):
        candidates = []
        jobs = []
        for sample in self.sample_batch:
            test_weights = self._test_weights(args, opt_graph, sample.optgraph_id)
            if len(test_weights) > 0:
                jobs.append((sample, test_weights))
        # the hyperbolic fits of every population member: independent small least-squares problems, fanned
        # out over a process pool when there are many (the reference forks per candidate in 3-D,
        # population_3d.py:216-237); results are the same function's, in job order
        preds = predict_all(args, opt_graph, [(s.optgraph_id, tw) for s, tw in jobs], self.bounded_search)
        for (sample, test_weights), res in zip(jobs, preds):
            for w, pred in zip(test_weights, res['predictions']):
                candidates.append({'sample': sample, 'weight': w, 'prediction': pred})

        virtual_ep = np.array([np.asarray(s.objs, dtype=np.float64) for s in ep.sample_batch]).reshape(-1, args.obj_num)
        mask = np.ones(len(candidates), dtype=bool)
        predicted_offspring_objs, elite_batch, scalarization_batch = [], [], []
        alpha = args.sparsity
        pred_arr = np.array([c['prediction'] for c in candidates], dtype=np.float64).reshape(-1, args.obj_num)
        for _ in range(args.num_tasks):
            best_id = self._best_candidate(virtual_ep, pred_arr, mask, alpha)
            if best_id == -1:
                print('Too few candidates')
                break
            c = candidates[best_id]
            elite_batch.append(c['sample'])
            sc = deepcopy(scalarization_template)
            sc.update_weights(c['weight'] / np.sum(c['weight']))
            scalarization_batch.append(sc)
            mask[best_id] = False
            virtual_ep = self._virtual_insert(virtual_ep, c['prediction'])
            predicted_offspring_objs.append(np.array(c['prediction'], dtype=np.float64))
        return elite_batch, scalarization_batch, predicted_offspring_objs

    def _best_candidate(self, virtual_ep, preds, mask, alpha):
        """First index of the maximum of HV - alpha * sparsity over the unmasked candidates (strict > scan in
        index order, population_2d.py:276-292), or -1."""
        best_id, best = -1, -np.inf
        for i in np.nonzero(mask)[0]:
            hv, sp = self._evaluate(virtual_ep, preds[i])
            if hv - alpha * sp > best:
                best, best_id = hv - alpha * sp, int(i)
        return best_id


class Population2d(_PopulationBase):
    """morl/population_2d.py:123-319."""

    def __init__(self, args):
        self.pbuffer_num = args.pbuffer_num
        self.dtheta = np.pi / 2.0 / self.pbuffer_num
        super().__init__(args)

    def insert_pbuffer(self, index, objs):
        """population_2d.py:141-167: bucket by the angle to the obj1 axis, keep the farthest."""
        f = np.asarray(objs, dtype=np.float64) - self.z_min
        if np.min(f) < 1e-7:
            return False
        dist = np.linalg.norm(f)
        theta = np.arccos(np.clip(f[1] / dist, -1.0, 1.0))
        buffer_id = int(theta // self.dtheta)
        if buffer_id < 0 or buffer_id >= self.pbuffer_num:
            return False
        return self._insert_sorted(buffer_id, index, dist)

    def _test_weights(self, args, opt_graph, node):
        """population_2d.py:238-258: num_weights directions evenly over ±pi/4 of the last weight,
        first quadrant only, minus directions already taken from this node."""
        num_weights = args.num_weight_candidates
        center = opt_graph.weights[node]
        ac = np.arctan2(center[1], center[0])
        lo, hi = ac - np.pi / 4., ac + np.pi / 4.
        succ_w = [opt_graph.weights[s] / np.linalg.norm(opt_graph.weights[s]) for s in opt_graph.succ[node]]
        out = []
        for i in range(num_weights):
            angle = lo + (hi - lo) / (num_weights - 1) * i
            w = np.array([np.cos(angle), np.sin(angle)])
            if w[0] >= -1e-7 and w[1] >= -1e-7 and not any(np.linalg.norm(s - w) < 1e-3 for s in succ_w):
                out.append(w)
        return out

    def compute_hypervolume(self, objs_batch):
        objs = np.asarray(objs_batch, dtype=np.float64)
        return _hv_2d_staircase(objs[get_ep_indices(objs)])

    def compute_sparsity(self, objs_batch):
        objs = np.asarray(objs_batch, dtype=np.float64)
        return _sparsity_ep_order(objs[get_ep_indices(objs)])

    def _evaluate(self, virtual_ep, pred):
        new = np.vstack([virtual_ep, np.asarray(pred, dtype=np.float64)[None]])
        e = new[get_ep_indices(new)]
        return _hv_2d_staircase(e), _sparsity_ep_order(e)

    def _best_candidate(self, virtual_ep, preds, mask, alpha):
        """Same result as the exact scan, fast: every candidate's score is first computed vectorised (the new
        front = virtual EP minus the points the candidate dominates, plus the candidate, in obj0 order) with a
        different float summation order; only the candidates within a rounding bound of the best screened
        score are then re-scored with the exact reference computation, scanned in index order with the strict
        > of the reference.  A candidate outside the bound scores below the best exactly, so the pick and
        its first-max tie-breaking are the reference's."""
        idx = np.nonzero(mask)[0]
        if len(idx) == 0:
            return -1
        score, mag = _screen_2d(virtual_ep, preds[idx], alpha)
        if np.isnan(score).all():  # every score NaN: no strict > ever holds (population_2d.py:286)
            return -1
        top = np.nanmax(score)
        tol = 1e-9 * (np.max(mag) + 1.0)
        near = idx[score >= top - 2.0 * tol]
        return _PopulationBase._best_candidate(self, virtual_ep, preds, np.isin(np.arange(len(preds)), near), alpha)

    def _virtual_insert(self, virtual_ep, pred):
        new = np.vstack([virtual_ep, np.asarray(pred, dtype=np.float64)[None]])
        return new[get_ep_indices(new)]


class Population3d(_PopulationBase):
    """morl/population_3d.py:120-345."""
    bounded_search = True

    def __init__(self, args):
        vec = weight_grid(args.obj_num, 1.0 / (args.pbuffer_num - 1))
        self.pbuffer_vec = np.array([np.asarray(v) / np.linalg.norm(v) for v in vec])
        self.pbuffer_num = len(self.pbuffer_vec)
        super().__init__(args)

    def find_buffer_id(self, f):
        """population_3d.py:134-140: the buffer direction with the largest dot product (first max)."""
        return int(np.argmax(self.pbuffer_vec @ f))

    def insert_pbuffer(self, index, objs, enforce=False):
        """population_3d.py:142-177."""
        f = np.asarray(objs, dtype=np.float64) - self.z_min
        if np.min(f) < 1e-7:
            return False
        return self._insert_sorted(self.find_buffer_id(f), index, np.linalg.norm(f), enforce)

    def _test_weights(self, args, opt_graph, node):
        """population_3d.py:245-287: the last weight (unless already taken), then grid weights at
        half the delta in a shuffled order, within pi/4 of it and not already taken."""
        num_weights = args.num_weight_candidates
        center = opt_graph.weights[node] / np.sum(opt_graph.weights[node])
        grid = weight_grid(args.obj_num, args.delta_weight / 2.0)
        succ_w = [opt_graph.weights[s] / np.sum(opt_graph.weights[s]) for s in opt_graph.succ[node]]
        out = []
        if not any(np.linalg.norm(s - center) < 1e-3 for s in succ_w):
            out.append(center)
        idx = np.array([i for i in range(len(grid))])
        np.random.shuffle(idx)
        cn = np.linalg.norm(center)
        for i in idx:
            if len(out) >= num_weights:
                break
            w = np.asarray(grid[i], dtype=np.float64)
            if np.linalg.norm(w - center) < 1e-3:
                continue
            angle = np.arccos(np.clip(np.dot(center, w) / cn / np.linalg.norm(w), -1.0, 1.0))
            if angle < np.pi / 4.0 and not any(np.linalg.norm(s - w) < 1e-3 for s in succ_w):
                out.append(w)
        return out

    def _evaluate(self, virtual_ep, pred):
        return _evaluate_3d(virtual_ep, pred)

    def _best_candidate(self, virtual_ep, preds, mask, alpha):
        """The exact per-candidate scores, computed over the fit pool in chunks when there are many (the
        reference forks one process per candidate, population_3d.py:216-237); the strict > scan in index order
        then runs here on the returned (identical) values."""
        idx = np.nonzero(mask)[0]
        pool = _fit_pool() if len(idx) >= 64 else None
        if pool is None:
            return _PopulationBase._best_candidate(self, virtual_ep, preds, mask, alpha)
        nch = min(len(idx), 4 * pool._processes)
        chunks = [idx[i::nch] for i in range(nch)]
        outs = pool.map(_score_chunk_3d, [(virtual_ep, preds[ch]) for ch in chunks])
        hv = np.empty(len(preds))
        sp = np.empty(len(preds))
        for ch, out in zip(chunks, outs):
            hv[ch], sp[ch] = out[:, 0], out[:, 1]
        best_id, best = -1, -np.inf
        for i in idx:
            if hv[i] - alpha * sp[i] > best:
                best, best_id = hv[i] - alpha * sp[i], int(i)
        return best_id

    def _virtual_insert(self, virtual_ep, pred):
        return update_ep(virtual_ep, pred)


def make_population(args):
    """morl/morl.py:46-51."""
    if args.obj_num == 2:
        return Population2d(args)
    if args.obj_num > 2:
        return Population3d(args)
    raise NotImplementedError('PG-MORL needs at least 2 objectives')
