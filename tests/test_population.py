"""Performance-buffer population and prediction-guided task selection (pgmorl_amd.population) against the
loop restatement in oracle/population.py, plus known-answer checks of the pieces (morl/population_2d.py,
morl/population_3d.py, morl/utils.py:41-66)."""
import argparse

import numpy as np
import pytest

from oracle import pareto as ref_pareto
from oracle import population as ref
from pgmorl_amd import pareto, population
from pgmorl_amd.sample import WeightedSumScalarization


class _S:
    def __init__(self, objs, node=None):
        self.objs = np.asarray(objs, dtype=np.float64)
        self.optgraph_id = node


class _EP:
    def __init__(self, samples):
        self.sample_batch = samples


def _args(K, **kw):
    a = dict(obj_num=K, num_tasks=5, num_weight_candidates=7, sparsity=1.0, delta_weight=0.2 if K == 2 else 0.25,
             pbuffer_num=100 if K == 2 else 20, pbuffer_size=2, min_weight=0.0, max_weight=1.0)
    a.update(kw)
    return argparse.Namespace(**a)


def _history(K, seed, gens=3):
    """A synthetic OptGraph: warm-up roots on the weight grid, then per generation one successor per leaf
    along a perturbed weight, improving roughly along that weight (what MOPG offspring look like)."""
    rng = np.random.RandomState(seed)
    og = pareto.OptGraph()
    grid = pareto.weight_grid(K, 0.2 if K == 2 else 0.25)
    leaves, offspring = [], []
    for w in grid:
        leaves.append(og.insert(np.asarray(w) + 1e-3, 20 + 10 * rng.rand(K), -1))
    for _ in range(gens):
        new = []
        for leaf in leaves:
            for _ in range(2):
                w = np.abs(og.weights[leaf] + 0.3 * rng.randn(K)) + 1e-3
                w = w / w.sum()
                objs = og.objs[leaf] + 40 * w + 3 * rng.randn(K) + 2
                node = og.insert(w, np.maximum(objs, 0.5), leaf)
                new.append(node)
                offspring.append(_S(og.objs[node], node))
        leaves = new
    return og, offspring


def test_population2d_buffers_known_answer():
    """Angular buffer bucketing and the per-buffer distance order (morl/population_2d.py:169-183)."""
    pop = population.Population2d(_args(2, pbuffer_num=4, pbuffer_size=2))
    # angle to the obj1 axis: buckets of pi/8; bucket 0 holds points near the obj1 axis
    pts = [(0.1, 5.0), (0.2, 9.0), (0.05, 1.0), (5.0, 5.0), (9.0, 0.1), (3.0, -1.0), (0.0, 4.0), (4.0, 4.1)]
    pop.update([_S(p) for p in pts])
    got = [tuple(s.objs) for s in pop.sample_batch]
    # bucket 0 holds (0.2,9) > (0.1,5) > (0.05,1): the nearest is dropped (size 2); (0,4) has a zero
    # coordinate and (3,-1) a negative one, so neither enters any buffer
    assert (0.2, 9.0) == got[0] and (0.1, 5.0) == got[1] and (0.05, 1.0) not in got
    assert (0.0, 4.0) not in got and (3.0, -1.0) not in got
    assert set(got) == {(0.2, 9.0), (0.1, 5.0), (5.0, 5.0), (4.0, 4.1), (9.0, 0.1)}
    ora = ref.Population2d(4, 2)
    ora.update([_S(p) for p in pts])
    assert got == [tuple(s.objs) for s in ora.sample_batch]


def test_population3d_buffer_directions():
    """The 3-D grid-direction buffers (morl/population_3d.py:122-125): 210 of them for --pbuffer-num 20 (the
    Hopper-v3 reading of SURVEY.md §8(d)), and find_buffer_id equal to the loop restatement."""
    pop = population.Population3d(_args(3, pbuffer_num=20))
    assert pop.pbuffer_num == 210
    ora = ref.Population3d(3, 20, 2)
    rng = np.random.RandomState(1)
    for f in rng.rand(200, 3):
        assert pop.find_buffer_id(f) == ora.buffer_id(f)


@pytest.mark.parametrize('K,seed', [(2, 0), (2, 1), (3, 0), (3, 1)])
def test_population_update_matches_oracle(K, seed):
    _, offspring = _history(K, seed)
    a = population.make_population(_args(K, pbuffer_num=10 if K == 2 else 6))
    b = ref.Population2d(10, 2) if K == 2 else ref.Population3d(3, 6, 2)
    for chunk in (offspring[:10], offspring[10:25], offspring[25:]):
        a.update(chunk)
        b.update(chunk)
        assert [id(s) for s in a.sample_batch] == [id(s) for s in b.sample_batch]


def test_predict_hyperbolic_recovers_a_known_curve():
    """Successor deltas drawn from f(w) = A tanh(a (w - b) / 2) + c per objective: the soft-L1 fit
    predicts f at unseen weights."""
    og = pareto.OptGraph()
    root = og.insert(np.array([0.5, 0.5]), np.array([100.0, 100.0]), -1)
    A, a, b, c = 30.0, 6.0, 0.5, 5.0
    f = lambda x: A * (np.exp(a * (x - b)) - 1) / (np.exp(a * (x - b)) + 1) + c  # noqa: E731
    for w0 in np.linspace(0.05, 0.95, 9):
        w = np.array([w0, 1 - w0])
        og.insert(w, og.objs[root] + np.array([f(w0), f(1 - w0)]), root)
    args = _args(2)
    test_w = [np.array([0.3, 0.7]), np.array([0.62, 0.38])]
    res = population.predict_hyperbolic(args, og, root, test_w)
    for w, p in zip(test_w, res['predictions']):
        np.testing.assert_allclose(p - og.objs[root], [f(w[0]), f(w[1])], rtol=0, atol=0.5)
    want = ref.predict_hyperbolic(2, og, root, test_w, three_d=False)
    np.testing.assert_allclose(np.array(res['predictions']), np.array(want), rtol=1e-9, atol=1e-9)


@pytest.mark.timeout(30)
def test_predict_hyperbolic_2d_terminates_with_few_weights():
    """population_2d.py:37-54 spins forever below four distinct weights; here it stops and still fits."""
    og = pareto.OptGraph()
    root = og.insert(np.array([0.5, 0.5]), np.array([10.0, 10.0]), -1)
    og.insert(np.array([0.3, 0.7]), np.array([12.0, 15.0]), root)
    og.insert(np.array([0.7, 0.3]), np.array([15.0, 11.0]), root)
    res = population.predict_hyperbolic(_args(2), og, root, [np.array([0.5, 0.5])])
    assert np.isfinite(res['predictions'][0]).all()
    lone = pareto.OptGraph()
    n = lone.insert(np.array([1.0, 1.0]), np.array([3.0, 4.0]), -1)   # no successor anywhere
    res = population.predict_hyperbolic(_args(2), lone, n, [np.array([0.5, 0.5])])
    np.testing.assert_array_equal(res['predictions'][0], [3.0, 4.0])


@pytest.mark.parametrize('K,seed', [(2, 0), (2, 3), (3, 0), (3, 2)])
def test_prediction_guided_selection_matches_oracle(K, seed):
    og, offspring = _history(K, seed)
    args = _args(K, pbuffer_num=10 if K == 2 else 6, num_tasks=6, sparsity=0.5)
    pop = population.make_population(args)
    pop.update(offspring)
    objs = np.array([s.objs for s in offspring])
    ep = _EP([offspring[i] for i in pareto.get_ep_indices(objs)])
    template = WeightedSumScalarization(num_objs=K, weights=np.ones(K) / K)
    np.random.seed(seed)
    elites, scal, preds = pop.prediction_guided_selection(args, 0, ep, og, template)
    ora = ref.Population2d(10, 2) if K == 2 else ref.Population3d(3, 6, 2)
    ora.update(offspring)
    ep_objs = [s.objs for s in ep.sample_batch]
    np.random.seed(seed)
    want = (ora.select(args.num_tasks, args.num_weight_candidates, args.sparsity, ep_objs, og) if K == 2 else
            ora.select(K, args.num_tasks, args.num_weight_candidates, args.delta_weight, args.sparsity, ep_objs, og))
    assert len(elites) == len(want) == args.num_tasks
    assert [e.optgraph_id for e in elites] == [s.optgraph_id for s, _, _ in want]
    for sc, (_, w, p), pr in zip(scal, want, preds):
        np.testing.assert_allclose(sc.weights.numpy(), w, rtol=0, atol=1e-12)
        assert sc.weights.sum().item() == pytest.approx(1.0, abs=1e-12)
        np.testing.assert_allclose(pr, p, rtol=1e-8, atol=1e-8)


def test_first_pick_is_the_best_hv_minus_alpha_sparsity():
    """The greedy step picks the candidate whose virtual insertion maximises HV - alpha * sparsity
    (population_2d.py:276-290), checked by brute force with the oracle's exact hypervolume."""
    og, offspring = _history(2, 5)
    args = _args(2, pbuffer_num=10, num_tasks=1, sparsity=0.0)
    pop = population.make_population(args)
    pop.update(offspring)
    objs = np.array([s.objs for s in offspring])
    ep = _EP([offspring[i] for i in pareto.get_ep_indices(objs)])
    elites, scal, preds = pop.prediction_guided_selection(args, 0, ep, og, WeightedSumScalarization(2, [0.5, 0.5]))
    base = np.array([s.objs for s in ep.sample_batch])
    best = -np.inf
    for s in pop.sample_batch:
        tw = pop._test_weights(args, og, s.optgraph_id)
        for p in population.predict_hyperbolic(args, og, s.optgraph_id, tw)['predictions'] if tw else []:
            new = np.vstack([base, p])
            best = max(best, ref_pareto._hv_max(new[ref_pareto.get_ep_indices(new)]))
    new = np.vstack([base, preds[0]])
    assert ref_pareto._hv_max(new[ref_pareto.get_ep_indices(new)]) == pytest.approx(best, rel=1e-12)


def test_random_selection_uses_the_global_stream():
    _, offspring = _history(2, 0)
    args = _args(2, pbuffer_num=10, num_tasks=4)
    pop = population.make_population(args)
    pop.update(offspring)
    t = WeightedSumScalarization(2, [0.5, 0.5])
    np.random.seed(7)
    e1, s1 = pop.random_selection(args, t)
    np.random.seed(7)
    want = []
    for _ in range(4):
        i = np.random.choice(len(pop.sample_batch))
        w = np.random.uniform(0.0, 1.0, 2)
        want.append((i, w / w.sum()))
    assert [id(e) for e in e1] == [id(pop.sample_batch[i]) for i, _ in want]
    for sc, (_, w) in zip(s1, want):
        np.testing.assert_array_equal(sc.weights.numpy(), w)
