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

Generation-boundary path in C++ (libpgm_host.so, include/pgm_host.h):
  * the soft-L1 hyperbolic fits of all population members run as one batch over the host's threads, a
    restatement of scipy's bounded 'trf' least_squares (the reference's call, population_2d.py:106);
  * the greedy knapsack (every round scores every candidate's virtual insertion: staircase HV / EP-order
    sparsity in 2-D, update_ep + hypervolume + utils.compute_sparsity in 3-D, strict > in index order) runs
    whole in one native call, the 3-D scoring threaded over candidates (the reference forks one process per
    candidate, population_3d.py:216-237).
The Python here keeps the reference's candidate construction (test weights, np.random draws, the
neighbourhood search) and the Population API.

Deliberate differences (documented in DESIGN.md):
  * The 3-D hypervolume sums slabs in an order of its own (rounded to 4 dp like hypervolume.py:74).
  * Fits agree with scipy's to ~1e-9 when they converge; fits that exhaust max_nfev (ill-conditioned,
    e.g. a slope at its bound) may stop at a slightly different point (tests/test_host_native.py).
  * The 2-D neighbourhood search (population_2d.py:37-54) has no exit when fewer than four
    distinct weights are reachable and spins forever; here it stops once a larger threshold
    cannot add any node.  When no node is reachable at all (the reference raises inside
    ``np.max`` of an empty array), the prediction is the unchanged objective vector.
  * scipy is the container's (1.15) rather than the pinned 1.4.1 (environment.yml:103): the
    fitted parameters are parity-unpinned beyond the tests' synthetic recoveries.
"""
from copy import deepcopy

import numpy as np

from . import _host
from .pareto import get_ep_indices, weight_grid

# --------------------------------------------------------------------------- prediction model


def collect_nearest_data(opt_graph, optgraph_id, threshold=0.1, objs_arr=None, edges=None):
    """population_2d.py:11-21: (objs, sum-normalised next weight, delta objs) of every successor
    edge leaving a node within ``threshold`` (relative, per objective) of node ``optgraph_id``, in the
    reference's order (parents ascending, each parent's successors in insertion order).
    ``objs_arr`` = np.array(opt_graph.objs) and ``edges`` = _edge_table(opt_graph), when the caller holds them."""
    objs_arr = np.asarray(opt_graph.objs, dtype=np.float64) if objs_arr is None else objs_arr
    parent, wn, dl = (_edge_table(opt_graph) if edges is None else edges)[:3]
    center = objs_arr[optgraph_id]
    near = np.all(np.abs(center - objs_arr) < np.abs(center) * threshold, axis=1)
    sel = near[parent]
    return objs_arr[parent[sel]], wn[sel], dl[sel]


def _edge_table(opt_graph):
    """Every OptGraph edge (parent, child) ordered by parent then child id (= each succ list's insertion
    order): the parents, the children's sum-normalised weights and their delta objs, as arrays."""
    par = np.asarray(opt_graph.prev, dtype=np.int64)
    child = np.nonzero(par >= 0)[0]
    parent = par[child]
    order = np.lexsort((child, parent))
    child, parent = child[order], parent[order]
    K = len(opt_graph.objs[0]) if len(opt_graph.objs) else 0
    W = np.asarray(opt_graph.weights, dtype=np.float64).reshape(-1, K)
    D = np.asarray(opt_graph.delta_objs, dtype=np.float64).reshape(-1, K)
    wn = W[child] / W[child].sum(axis=1, keepdims=True)
    has_succ = np.zeros(len(par), dtype=bool)
    has_succ[parent] = True
    return parent, wn, D[child], has_succ


def _count_distinct(weights_data, enough=4):
    """population_2d.py:39-44: weights i with every earlier weight j at distance >= 1e-5, counted up to
    ``enough`` (one vectorised distance row per i instead of the reference's pair loop; same predicate)."""
    W = np.asarray(weights_data, dtype=np.float64)
    cnt = 0
    for i in range(len(W)):
        if i == 0 or bool(np.all(np.linalg.norm(W[i] - W[:i], axis=1) >= 1e-5)):
            cnt += 1
            if cnt >= enough:
                break
    return cnt


def _max_useful_threshold(opt_graph, optgraph_id, objs_arr, has_succ=None):
    """Smallest threshold beyond which collect_nearest_data cannot grow any more (nodes relative to a
    centre with a zero coordinate need diff < 0 there: never reachable)."""
    center = np.abs(objs_arr[optgraph_id])
    if np.any(center == 0):
        return 0.0
    if has_succ is None:
        has_succ = np.array([len(s) > 0 for s in opt_graph.succ])
    if not has_succ.any():
        return 0.0
    diff = np.abs(objs_arr[optgraph_id] - objs_arr[has_succ])
    return float(np.max(diff / center))


def _hyperbolic(x, A, a, b, c):
    e = np.exp(a * (x - b))
    return A * (e - 1) / (e + 1) + c


def _fit_inputs(args, opt_graph, optgraph_id, test_weights, bounded_search, objs_arr, edges=None):
    """population_2d.py:27-104 / population_3d.py:23-97 up to the fits: the widening neighbourhood search, the
    Gaussian distance weights and one (x, y, w, A upper bound) fit problem per objective.  Returns
    (original objs, sum-normalised test weights, problems or None when no node is reachable)."""
    test_weights = np.array(test_weights, dtype=np.float64)
    test_weights = test_weights / test_weights.sum(axis=1, keepdims=True)
    threshold, sigma = 0.1, 0.03
    t_max = None if bounded_search else _max_useful_threshold(opt_graph, optgraph_id, objs_arr,
                                                              None if edges is None else edges[3])
    while True:
        objs_data, weights_data, delta_objs_data = collect_nearest_data(opt_graph, optgraph_id, threshold, objs_arr,
                                                                        edges)
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
        return original, test_weights, None
    objs_data = np.array(objs_data, dtype=np.float64)
    weights_data = np.array(weights_data, dtype=np.float64)
    delta_objs_data = np.array(delta_objs_data, dtype=np.float64)
    dist = np.linalg.norm(np.abs(objs_data - original) / np.abs(original), axis=1)
    w = np.exp(-((dist / sigma) ** 2) / 2.0)
    problems = []
    for dim in range(args.obj_num):
        x, y = weights_data[:, dim], delta_objs_data[:, dim]
        problems.append((x, y, w, float(np.clip(np.max(y) - np.min(y), 1.0, 500.0))))
    return original, test_weights, problems


def predict_all(args, opt_graph, jobs, bounded_search):
    """predict_hyperbolic for every (node, test_weights) job, in order.  The per-objective soft-L1 fits of all
    jobs (population_2d.py:105-113: least_squares(fun, ones(4), loss='soft_l1', f_scale=20, jac=jac,
    bounds=([0, .1, -5, -500], [A_hi, 20, 5, 500]))) run as ONE batch in libpgm_host.so (a C++ restatement of
    scipy's bounded 'trf' with the exact trust-region solver, over the host's threads)."""
    objs_arr = np.asarray(opt_graph.objs, dtype=np.float64)
    edges = _edge_table(opt_graph)
    prep = [_fit_inputs(args, opt_graph, node, tw, bounded_search, objs_arr, edges) for node, tw in jobs]
    problems = [p for _, _, probs in prep if probs is not None for p in probs]
    params = _host.fit_hyperbolic(problems) if problems else np.zeros((0, 4))
    out, k = [], 0
    for (node, _), (original, tw, probs) in zip(jobs, prep):
        if probs is None:  # nothing reachable: the prediction is the unchanged objective vector
            out.append({'sample_index': node, 'predictions': [original.copy() for _ in range(len(tw))]})
            continue
        deltas = np.array([_hyperbolic(tw.T[dim], *params[k + dim]) for dim in range(args.obj_num)]).T
        k += args.obj_num
        out.append({'sample_index': node, 'predictions': [original + deltas[i] for i in range(len(tw))]})
    return out


def predict_hyperbolic(args, opt_graph, optgraph_id, test_weights, bounded_search=False):
    """population_2d.py:27-118 (bounded_search=False) / population_3d.py:23-112 (True, which adds the
    ``threshold >= 1.0`` exit of population_3d.py:46)."""
    return predict_all(args, opt_graph, [(optgraph_id, test_weights)], bounded_search)[0]


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
        # the hyperbolic fits of every population member: independent small least-squares problems, one
        # native batch (the reference fits them one after another)
        preds = predict_all(args, opt_graph, [(s.optgraph_id, tw) for s, tw in jobs], self.bounded_search)
        for (sample, test_weights), res in zip(jobs, preds):
            for w, pred in zip(test_weights, res['predictions']):
                candidates.append({'sample': sample, 'weight': w, 'prediction': pred})

        virtual_ep = np.array([np.asarray(s.objs, dtype=np.float64) for s in ep.sample_batch]).reshape(-1, args.obj_num)
        pred_arr = np.array([c['prediction'] for c in candidates], dtype=np.float64).reshape(-1, args.obj_num)
        picks = _host.select_greedy(virtual_ep, pred_arr, args.sparsity, args.num_tasks, self.select_mode)
        if len(picks) < args.num_tasks:
            print('Too few candidates')
        predicted_offspring_objs, elite_batch, scalarization_batch = [], [], []
        for best_id in picks:
            c = candidates[best_id]
            elite_batch.append(c['sample'])
            sc = deepcopy(scalarization_template)
            sc.update_weights(c['weight'] / np.sum(c['weight']))
            scalarization_batch.append(sc)
            predicted_offspring_objs.append(np.array(c['prediction'], dtype=np.float64))
        return elite_batch, scalarization_batch, predicted_offspring_objs


class Population2d(_PopulationBase):
    """morl/population_2d.py:123-319."""
    select_mode = _host.STAIRCASE

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
        succ_w = _rows([opt_graph.weights[s] / np.linalg.norm(opt_graph.weights[s]) for s in opt_graph.succ[node]], 2)
        out = []
        for i in range(num_weights):
            angle = lo + (hi - lo) / (num_weights - 1) * i
            w = np.array([np.cos(angle), np.sin(angle)])
            if w[0] >= -1e-7 and w[1] >= -1e-7 and not _taken(succ_w, w):
                out.append(w)
        return out

    def compute_hypervolume(self, objs_batch):
        """population_2d.py:185-192: staircase over the EP (ascending obj0), reference point (0, 0)."""
        objs = np.asarray(objs_batch, dtype=np.float64)
        hv, x = 0.0, 0.0
        for o in objs[get_ep_indices(objs)]:
            hv += (max(0.0, o[0]) - x) * (max(0.0, o[1]) - 0.0)
            x = max(0.0, o[0])
        return hv

    def compute_sparsity(self, objs_batch):
        """population_2d.py:194-202: mean squared step between consecutive EP points."""
        objs = np.asarray(objs_batch, dtype=np.float64)
        e = objs[get_ep_indices(objs)]
        if len(e) < 2:
            return 0.0
        sp = 0.0
        for i in range(1, len(e)):
            sp += np.sum(np.square(e[i] - e[i - 1]))
        return sp / (len(e) - 1)


class Population3d(_PopulationBase):
    """morl/population_3d.py:120-345."""
    bounded_search = True
    select_mode = _host.UPDATE_EP

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
        succ_w = _rows([opt_graph.weights[s] / np.sum(opt_graph.weights[s]) for s in opt_graph.succ[node]], args.obj_num)
        out = []
        if not _taken(succ_w, center):
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
            if angle < np.pi / 4.0 and not _taken(succ_w, w):
                out.append(w)
        return out


def _rows(ws, k):
    return np.array(ws, dtype=np.float64).reshape(-1, k)


def _taken(succ_w, w):
    """any(np.linalg.norm(s - w) < 1e-3 for s in succ_w) over the rows at once (population_2d.py:253-255,
    population_3d.py:270-283): the direction w was already taken from this node."""
    if not len(succ_w):
        return False
    d = succ_w - w
    return bool(np.any(np.sqrt((d * d).sum(axis=1)) < 1e-3))


def make_population(args):
    """morl/morl.py:46-51."""
    if args.obj_num == 2:
        return Population2d(args)
    if args.obj_num > 2:
        return Population3d(args)
    raise NotImplementedError('PG-MORL needs at least 2 objectives')
