"""Oracle: performance-buffer population + prediction-guided selection, plain loops.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates, element by element:
  * update_ep                               -- morl/utils.py:41-66
  * collect_nearest_data / predict_hyperbolic (search loop, Gaussian weights, soft-L1 fit)
                                            -- morl/population_2d.py:11-118, population_3d.py:13-112
  * 2-D buffers, staircase HV, EP-order sparsity, +-pi/4 candidate fan, greedy knapsack
                                            -- morl/population_2d.py:123-304
  * 3-D buffers (grid directions), shuffled candidates, update_ep-based greedy
                                            -- morl/population_3d.py:114-333
The 2-D search stops when four distinct weights are found or the threshold passes 1e3 (the
reference has no exit there; the product stops as soon as no node can be added -- the tests only
use graphs where both exits agree).
"""
from copy import deepcopy

import numpy as np
from scipy.optimize import least_squares

from .pareto import compute_hypervolume, compute_sparsity, generate_weights_batch_dfs, get_ep_indices


def update_ep(ep_objs_batch, new_objs):
    if (np.asarray(new_objs) < 0).any():
        return deepcopy(list(ep_objs_batch))
    out, on_ep = [], True
    for p in ep_objs_batch:
        p = np.asarray(p)
        if (p >= new_objs - 1e-5).all() and (p > new_objs + 1e-5).any():
            on_ep = False
        if not (new_objs >= p).all():
            out.append(p.copy())
    if on_ep:
        for i in range(len(out)):
            if new_objs[0] < out[i][0]:
                out.insert(i, np.array(new_objs, copy=True))
                break
        else:
            out.append(np.array(new_objs, copy=True))
    return out


def predict_hyperbolic(obj_num, opt_graph, index, test_weights, three_d):
    tw = np.array(test_weights, dtype=np.float64)
    for row in tw:
        row /= np.sum(row)
    threshold, sigma = 0.1, 0.03
    while True:
        od, wd, dd = [], [], []
        for i in range(len(opt_graph.objs)):
            if np.all(np.abs(opt_graph.objs[index] - opt_graph.objs[i]) < np.abs(opt_graph.objs[index]) * threshold):
                for n in opt_graph.succ[i]:
                    od.append(opt_graph.objs[i])
                    wd.append(opt_graph.weights[n] / np.sum(opt_graph.weights[n]))
                    dd.append(opt_graph.delta_objs[n])
        cnt = 0
        for i in range(len(wd)):
            if all(np.linalg.norm(wd[i] - wd[j]) >= 1e-5 for j in range(i)):
                cnt += 1
                if cnt > 3:
                    break
        if cnt > 3 or (three_d and threshold >= 1.0) or (not three_d and threshold > 1e3):
            break
        threshold *= 2.0
        sigma *= 2.0

    preds = []
    for dim in range(obj_num):
        x = np.array([w[dim] for w in wd])
        y = np.array([d[dim] for d in dd])
        wt = np.array([np.exp(-((np.linalg.norm(np.abs(o - opt_graph.objs[index]) / np.abs(opt_graph.objs[index]))
                                 / sigma) ** 2) / 2.0) for o in od])

        def f(xx, A, a, b, c):
            return A * (np.exp(a * (xx - b)) - 1) / (np.exp(a * (xx - b)) + 1) + c

        def fun(p, xx, yy):
            return (f(xx, *p) - yy) * wt

        def jac(p, xx, yy):
            A, a, b, _ = p
            e = np.exp(a * (xx - b))
            return np.stack([(e - 1) / (e + 1) * wt, A * (xx - b) * 2. * e / (e + 1) ** 2 * wt,
                             A * (-a) * 2. * e / (e + 1) ** 2 * wt, wt]).T

        hi = np.clip(np.max(y) - np.min(y), 1.0, 500.0)
        r = least_squares(fun, np.ones(4), loss='soft_l1', f_scale=20., args=(x, y), jac=jac,
                          bounds=([0, 0.1, -5., -500.], [hi, 20., 5., 500.]))
        preds.append(f(tw.T[dim], *r.x))
    preds = np.array(preds).T
    return [opt_graph.objs[index] + preds[i] for i in range(len(tw))]


class Population2d:
    def __init__(self, pbuffer_num, pbuffer_size):
        self.pbuffer_num, self.pbuffer_size = pbuffer_num, pbuffer_size
        self.dtheta = np.pi / 2.0 / pbuffer_num
        self.sample_batch = []

    def _bucket(self, f):
        dist = np.linalg.norm(f)
        return int(np.arccos(np.clip(f[1] / dist, -1.0, 1.0)) // self.dtheta), dist

    def update(self, samples):
        allb = self.sample_batch + list(samples)
        bufs = [[] for _ in range(self.pbuffer_num)]
        dists = [[] for _ in range(self.pbuffer_num)]
        for idx, s in enumerate(allb):
            f = np.asarray(s.objs, dtype=np.float64)
            if np.min(f) < 1e-7:
                continue
            b, d = self._bucket(f)
            if b < 0 or b >= self.pbuffer_num:
                continue
            pos = next((i for i in range(len(bufs[b])) if dists[b][i] < d), None)
            if pos is not None:
                bufs[b].insert(pos, idx)
                dists[b].insert(pos, d)
                bufs[b], dists[b] = bufs[b][:self.pbuffer_size], dists[b][:self.pbuffer_size]
            elif len(bufs[b]) < self.pbuffer_size:
                bufs[b].append(idx)
                dists[b].append(d)
        self.sample_batch = [allb[i] for b in bufs for i in b]

    @staticmethod
    def _hv(objs):
        e = np.array(objs)[get_ep_indices(objs)]
        hv, x = 0.0, 0.0
        for o in e:
            hv += (max(0.0, o[0]) - x) * max(0.0, o[1])
            x = max(0.0, o[0])
        return hv

    @staticmethod
    def _sp(objs):
        e = np.array(objs)[get_ep_indices(objs)]
        if len(e) < 2:
            return 0.0
        return sum(np.sum(np.square(e[i] - e[i - 1])) for i in range(1, len(e))) / (len(e) - 1)

    def select(self, num_tasks, num_weights, alpha, ep_objs, opt_graph):
        cands = []
        for s in self.sample_batch:
            c = opt_graph.weights[s.optgraph_id]
            ac = np.arctan2(c[1], c[0])
            tws = []
            for i in range(num_weights):
                ang = ac - np.pi / 4 + (np.pi / 2) / (num_weights - 1) * i
                w = np.array([np.cos(ang), np.sin(ang)])
                if w[0] >= -1e-7 and w[1] >= -1e-7:
                    if not any(np.linalg.norm(opt_graph.weights[n] / np.linalg.norm(opt_graph.weights[n]) - w) < 1e-3
                               for n in opt_graph.succ[s.optgraph_id]):
                        tws.append(w)
            if tws:
                for w, p in zip(tws, predict_hyperbolic(2, opt_graph, s.optgraph_id, tws, False)):
                    cands.append((s, w, p))
        vep = [np.array(o) for o in ep_objs]
        mask = [True] * len(cands)
        out = []
        for _ in range(num_tasks):
            best, bid = -np.inf, -1
            for i, (_, _, p) in enumerate(cands):
                if mask[i]:
                    v = self._hv(vep + [p]) - alpha * self._sp(vep + [p])
                    if v > best:
                        best, bid = v, i
            if bid < 0:
                break
            s, w, p = cands[bid]
            out.append((s, w / np.sum(w), p))
            mask[bid] = False
            nb = np.array(vep + [p])
            vep = list(nb[get_ep_indices(nb)])
        return out


class Population3d:
    def __init__(self, obj_num, pbuffer_num, pbuffer_size):
        vec = []
        generate_weights_batch_dfs(0, obj_num, 0.0, 1.0, 1.0 / (pbuffer_num - 1), [], vec)
        self.vec = [np.array(v) / np.linalg.norm(v) for v in vec]
        self.pbuffer_size = pbuffer_size
        self.sample_batch = []

    def buffer_id(self, f):
        best, bid = -np.inf, -1
        for i, v in enumerate(self.vec):
            d = np.dot(v, f)
            if d > best:
                best, bid = d, i
        return bid

    def update(self, samples):
        allb = self.sample_batch + list(samples)
        bufs = [[] for _ in self.vec]
        dists = [[] for _ in self.vec]
        for idx, s in enumerate(allb):
            f = np.asarray(s.objs, dtype=np.float64)
            if np.min(f) < 1e-7:
                continue
            b, d = self.buffer_id(f), np.linalg.norm(f)
            pos = next((i for i in range(len(bufs[b])) if dists[b][i] < d), None)
            if pos is not None:
                bufs[b].insert(pos, idx)
                dists[b].insert(pos, d)
                bufs[b], dists[b] = bufs[b][:self.pbuffer_size], dists[b][:self.pbuffer_size]
            elif len(bufs[b]) < self.pbuffer_size:
                bufs[b].append(idx)
                dists[b].append(d)
        self.sample_batch = [allb[i] for b in bufs for i in b]

    def select(self, obj_num, num_tasks, num_weights, delta_weight, alpha, ep_objs, opt_graph):
        cands = []
        for s in self.sample_batch:
            c = opt_graph.weights[s.optgraph_id]
            c = c / np.sum(c)
            grid = []
            generate_weights_batch_dfs(0, obj_num, 0.0, 1.0, delta_weight / 2.0, [], grid)
            taken = [opt_graph.weights[n] / np.sum(opt_graph.weights[n]) for n in opt_graph.succ[s.optgraph_id]]
            tws = [] if any(np.linalg.norm(t - c) < 1e-3 for t in taken) else [c]
            order = np.array(list(range(len(grid))))
            np.random.shuffle(order)
            for i in order:
                if len(tws) >= num_weights:
                    break
                w = np.array(grid[i])
                if np.linalg.norm(w - c) < 1e-3:
                    continue
                ang = np.arccos(np.clip(np.dot(c, w) / np.linalg.norm(c) / np.linalg.norm(w), -1.0, 1.0))
                if ang < np.pi / 4.0 and not any(np.linalg.norm(t - w) < 1e-3 for t in taken):
                    tws.append(w)
            if tws:
                for w, p in zip(tws, predict_hyperbolic(obj_num, opt_graph, s.optgraph_id, tws, True)):
                    cands.append((s, w, p))
        vep = [np.array(o) for o in ep_objs]
        mask = [True] * len(cands)
        out = []
        for _ in range(num_tasks):
            best, bid = -np.inf, -1
            for i, (_, _, p) in enumerate(cands):
                if mask[i]:
                    e = update_ep(vep, p)
                    v = compute_hypervolume(e) - alpha * compute_sparsity(e)
                    if v > best:
                        best, bid = v, i
            if bid < 0:
                break
            s, w, p = cands[bid]
            out.append((s, w / np.sum(w), p))
            mask[bid] = False
            vep = update_ep(vep, p)
        return out
