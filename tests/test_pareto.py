"""Generation-boundary host logic (pgmorl_amd.pareto) against the oracle restatement: bit-exact EP
membership and order (north-star bar), hypervolume, sparsity, weight grids and OptGraph."""
import numpy as np
import pytest

from oracle import pareto as ref
from pgmorl_amd import pareto


def _fronts(seed, n, K):
    rng = np.random.RandomState(seed)
    x = rng.rand(n, K) * 10 - 0.5                    # a few negative points (never in the EP)
    x[: n // 5] = np.round(x[: n // 5], 1)            # ties
    if n > 4:
        x[1] = x[0]                                   # exact duplicates
        x[3, 0] = x[2, 0]                             # equal obj0 (argsort order matters)
    return x


@pytest.mark.parametrize('K', [2, 3])
@pytest.mark.parametrize('seed', range(6))
def test_ep_indices_bit_exact(K, seed):
    for n in (0, 1, 2, 7, 64, 300):
        x = _fronts(seed, n, K)
        assert list(pareto.get_ep_indices(x)) == list(ref.get_ep_indices(x))


class _S:
    def __init__(self, objs):
        self.objs = objs


def test_ep_update_sequence_matches_oracle():
    rng = np.random.RandomState(3)
    a, b = pareto.EP(), ref.EP()
    for gen in range(6):
        batch = [_S(o) for o in rng.rand(25, 2) * (gen + 1)]
        a.update(batch)
        b.update(batch)
        np.testing.assert_array_equal(a.obj_batch, b.obj_batch)
        assert [id(s) for s in a.sample_batch] == [id(s) for s in b.sample_batch]


@pytest.mark.parametrize('K', [2, 3])
def test_hypervolume_and_sparsity(K):
    for seed in range(5):
        x = np.abs(_fronts(seed, 40, K))
        front = x[pareto.get_ep_indices(x)]
        assert pareto.compute_hypervolume(front) == ref.compute_hypervolume(front)
        assert pareto.compute_sparsity(front) == pytest.approx(ref.compute_sparsity(front), rel=1e-12)
    if K == 2:  # 2-D sweep of scripts/plot/ep_batch_visualize_2d.py on a non-dominated front
        hv, _ = ref.hv_sparsity_2d(front)
        assert pareto.compute_hypervolume(front) == pytest.approx(round(hv, 4), abs=1e-4)
    assert pareto.compute_hypervolume(np.zeros((0, K))) == 0.0


@pytest.mark.parametrize('obj_num,delta,count', [(2, 0.25, 5), (2, 1 / 39, 40), (2, 1 / 159, 160),
                                                 (3, 1 / 19, 210), (2, 0.2, 6)])
def test_weight_grids(obj_num, delta, count):
    got = pareto.weight_grid(obj_num, delta)
    want = []
    ref.generate_weights_batch_dfs(0, obj_num, 0.0, 1.0, delta, [], want)
    assert len(got) == count
    np.testing.assert_array_equal(np.array(got), np.array(want))


def test_optgraph_matches_oracle():
    a, b = pareto.OptGraph(), ref.OptGraph()
    rng = np.random.RandomState(0)
    prev_a = prev_b = -1
    for i in range(10):
        w, o = rng.rand(2), rng.rand(2)
        prev_a, prev_b = a.insert(w, o, prev_a if i % 3 else -1), b.insert(w, o, prev_b if i % 3 else -1)
        assert prev_a == prev_b
    for f in ('weights', 'objs', 'delta_objs'):
        np.testing.assert_array_equal(np.array(getattr(a, f)), np.array(getattr(b, f)))
    assert a.prev == b.prev and a.succ == b.succ
