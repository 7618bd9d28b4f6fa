"""Host profile of the generation boundary (morl/morl.py:100-175) at pop=40 scale without a GPU: a synthetic
MOPG stand-in (offspring objectives drift along the task weight, like _history in tests/test_population.py)
feeds the real EP / population / OptGraph / prediction-guided selection of pgmorl_amd, and every piece is
timed.  Usage: python scripts/prof_boundary.py [generations]"""
import argparse
import os
import sys
import time
from copy import deepcopy

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from pgmorl_amd import pareto
from pgmorl_amd.population import make_population
from pgmorl_amd.sample import WeightedSumScalarization


class _S:
    def __init__(self, objs, node=-1):
        self.objs = np.asarray(objs, dtype=np.float64)
        self.optgraph_id = node


def main(gens=6, K=2, P=40, iters=20, seed=0):
    rng = np.random.RandomState(seed)
    args = argparse.Namespace(obj_num=K, num_tasks=P, num_weight_candidates=7, sparsity=1.0, pbuffer_num=100,
                              pbuffer_size=2, min_weight=0.0, max_weight=1.0, delta_weight=1.0 / (P - 1),
                              update_iter=iters, warmup_iter=4 * iters)
    ep, og, pop = pareto.EP(), pareto.OptGraph(), make_population(args)
    tmpl = WeightedSumScalarization(num_objs=K, weights=np.ones(K) / K)
    grid = pareto.weight_grid(K, args.delta_weight)
    elites = [_S(200 + 50 * rng.rand(K)) for _ in grid]
    scal = []
    for e, w in zip(elites, grid):
        e.optgraph_id = og.insert(np.asarray(w), e.objs, -1)
        sc = deepcopy(tmpl)
        sc.update_weights(w)
        scal.append(sc)
    tot = {}

    def tick(k, t0):
        tot[k] = tot.get(k, 0.0) + time.perf_counter() - t0
        return time.perf_counter()

    n_its = args.warmup_iter
    for gen in range(gens):
        t = time.perf_counter()
        all_samples, offspring = [], []
        for e, sc in zip(elites, scal):
            w = sc.weights.numpy()
            prev, objs = e.optgraph_id, e.objs.copy()
            for i in range(n_its):
                objs = objs + 2.0 * w * rng.rand() + 0.5 * rng.randn(K)
                s = _S(objs.copy())
                all_samples.append(s)
                if (i + 1) % iters == 0:
                    prev = og.insert(w, objs.copy(), prev)
                    s.optgraph_id = prev
                    offspring.append(s)
        t = tick('mopg stand-in', t)
        ep.update(all_samples)
        t = tick('ep.update', t)
        pop.update(offspring)
        t = tick('population.update', t)
        elites, scal, _ = pop.prediction_guided_selection(args, gen, ep, og, tmpl)
        t = tick('prediction_guided_selection', t)
        n_its = iters
        print(f'gen {gen}: ep {len(ep.obj_batch)} pop {len(pop.sample_batch)} nodes {len(og.objs)} '
              f'tasks {len(elites)} | ' + ', '.join(f'{k} {v:.2f}s' for k, v in tot.items()), flush=True)
    return tot


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 6)
