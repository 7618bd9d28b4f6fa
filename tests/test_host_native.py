"""libpgm_host.so (include/pgm_host.h): the native generation-boundary path against its checkers.

  * pgm_fit_hyperbolic vs scipy.optimize.least_squares itself (the reference's call, morl/population_2d.py:106:
    loss='soft_l1', f_scale=20, the analytic Jacobian, bounds [0, .1, -5, -500] .. [A_hi, 20, 5, 500]) on
    problems shaped like the selection's (weights in [0, 1], Gaussian sample weights, noisy hyperbolic deltas);
  * pgm_select_greedy vs the reference-order exact scans restated in oracle/population.py (2-D staircase) and
    oracle/population.update_ep + oracle/pareto.compute_hypervolume / compute_sparsity (update_ep mode), pick
    for pick, on candidate sets with exact ties, EP duplicates, dominated and negative predictions;
  * pgm_hypervolume / pgm_ep_mask vs oracle/pareto.
scipy is the container's 1.15.3 (the reference pins 1.4.1, environment.yml:103): the fits are pinned to that
scipy, not to the reference's own numbers (none exist for them)."""
import ctypes
import os
import re

import numpy as np
import pytest
from scipy.optimize import least_squares

from oracle import pareto as ref_pareto
from oracle import population as ref_pop
from pgmorl_amd import _host, pareto

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'include', 'pgm_host.h')


def test_library_exports_every_declared_symbol():
    names = re.findall(r'^\w[\w\s\*]*?\b(pgm_\w+)\(', open(HDR).read(), re.M)
    assert len(names) >= 6
    lib = ctypes.CDLL(_host.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    assert _host.lib().pgm_host_abi_version() == _host.PGM_HOST_ABI_VERSION


def _problems(seed, n):
    rng = np.random.RandomState(seed)
    out = []
    for _ in range(n):
        m = rng.randint(4, 60)
        x = rng.rand(m)
        A, a, b, c = rng.uniform(0, 50), rng.uniform(0.1, 20), rng.uniform(-1, 1), rng.uniform(-20, 20)
        e = np.exp(a * (x - b))
        y = A * (e - 1) / (e + 1) + c + rng.randn(m) * rng.choice([0.1, 5, 30])
        w = np.exp(-rng.rand(m) ** 2 * rng.choice([0.5, 5, 50]))
        out.append((x, y, w, float(np.clip(y.max() - y.min(), 1.0, 500.0))))
    return out


def _fun(p, x, y, w):
    e = np.exp(p[1] * (x - p[2]))
    return (p[0] * (e - 1.) / (e + 1) + p[3] - y) * w


def _jac(p, x, y, w):
    A, a, b, _ = p
    e = np.exp(a * (x - b))
    J = np.empty((4, len(x)))
    J[0] = (e - 1) / (e + 1) * w
    J[1] = A * (x - b) * (2. * e) / ((e + 1) ** 2) * w
    J[2] = A * (-a) * (2. * e) / ((e + 1) ** 2) * w
    J[3] = w
    return J.T


def _cost(p, x, y, w):
    z = (_fun(p, x, y, w) / 20.) ** 2
    return 0.5 * 400. * np.sum(2 * (np.sqrt(1 + z) - 1))


def test_fits_match_scipy_least_squares():
    probs = _problems(0, 160)
    got, nfev = _host.fit_hyperbolic(probs, return_nfev=True)
    xt = np.linspace(0, 1, 11)
    f = lambda x, p: p[0] * (np.exp(p[1] * (x - p[2])) - 1) / (np.exp(p[1] * (x - p[2])) + 1) + p[3]  # noqa: E731
    close, same_nfev = 0, 0
    for (x, y, w, ah), p, ne in zip(probs, got, nfev):
        r = least_squares(_fun, np.ones(4), loss='soft_l1', f_scale=20., args=(x, y, w), jac=_jac,
                          bounds=([0, 0.1, -5., -500.], [ah, 20., 5., 500.]))
        assert (p >= [0, 0.1, -5, -500]).all() and (p <= [ah, 20, 5, 500]).all()
        same_nfev += ne == r.nfev
        rel = np.abs(f(xt, p) - f(xt, r.x)).max() / (1 + np.abs(f(xt, r.x)).max())
        close += rel < 1e-6
        # where the two paths part (ill-conditioned fits that run to max_nfev), neither optimum is worse by more
        # than a hair
        assert rel < 2e-3
        assert _cost(p, x, y, w) <= _cost(r.x, x, y, w) * (1 + 2e-3) + 1e-9
    assert same_nfev >= 0.97 * len(probs)
    assert close >= 0.97 * len(probs)


def test_fit_threads_do_not_change_results():
    probs = _problems(1, 40)
    np.testing.assert_array_equal(_host.fit_hyperbolic(probs, nthreads=1), _host.fit_hyperbolic(probs, nthreads=7))


def test_fit_rejects_bad_input():
    with pytest.raises(_host.PGMHostError):
        _host.fit_hyperbolic([(np.zeros(0), np.zeros(0), np.zeros(0), 1.0)])
    with pytest.raises(_host.PGMHostError):
        _host.fit_hyperbolic([(np.ones(3), np.ones(3), np.ones(3), 0.0)])


# ---------------------------------------------------------------- greedy selection vs the exact reference scans
def _ref_sparsity(e):
    """morl/utils.py:87-100 in the reference's summation order (dimension-major, sorted, one running sum)."""
    if len(e) < 2:
        return 0.0
    sp = 0.0
    arr = np.array(e)
    for d in range(arr.shape[1]):
        col = np.sort(arr[:, d])
        for i in range(1, len(col)):
            sp += np.square(col[i] - col[i - 1])
    return sp / (len(e) - 1)


def _scan(ep, preds, alpha, n_pick, mode):
    vep = [np.array(o) for o in ep]
    mask = np.ones(len(preds), dtype=bool)
    out = []
    for _ in range(n_pick):
        best, bid = -np.inf, -1
        for i in range(len(preds)):
            if not mask[i]:
                continue
            if mode == _host.STAIRCASE:
                v = ref_pop.Population2d._hv(vep + [preds[i]]) - alpha * ref_pop.Population2d._sp(vep + [preds[i]])
            else:
                e = ref_pop.update_ep(vep, preds[i])
                v = (ref_pareto.compute_hypervolume(e) - alpha * _ref_sparsity(e)) if len(e) else 0.0
            if v > best:
                best, bid = v, i
        if bid < 0:
            break
        out.append(bid)
        mask[bid] = False
        if mode == _host.STAIRCASE:
            nb = np.array(vep + [preds[bid]])
            vep = list(nb[ref_pareto.get_ep_indices(nb)])
        else:
            vep = ref_pop.update_ep(vep, preds[bid])
    return out


def _cands(rng, K, n_ep, n_c, scale=100.0):
    ep = rng.rand(n_ep, K) * scale
    ep = ep[pareto.get_ep_indices(ep)] if n_ep else ep.reshape(0, K)
    preds = rng.rand(n_c, K) * (1.1 * scale) - 0.05 * scale
    preds[::7] = preds[3]  # exact ties: the first index wins
    if len(ep):
        preds[5::11] = ep[rng.randint(len(ep), size=len(preds[5::11]))]  # duplicates of EP points
    return ep, preds


@pytest.mark.parametrize('seed', range(6))
def test_greedy_staircase_equals_reference_scan(seed):
    rng = np.random.RandomState(seed)
    ep, preds = _cands(rng, 2, rng.randint(0, 40), 120)
    for alpha in (0.0, 1.0, 30.0):
        assert _host.select_greedy(ep, preds, alpha, 8, _host.STAIRCASE) == _scan(ep, preds, alpha, 8, _host.STAIRCASE)


@pytest.mark.parametrize('K,seed', [(2, 0), (2, 1), (3, 0), (3, 1), (3, 2)])
def test_greedy_update_ep_equals_reference_scan(K, seed):
    rng = np.random.RandomState(seed)
    ep, preds = _cands(rng, K, rng.randint(0, 30), 60 if K == 3 else 100, scale=50.0)
    for alpha in (0.0, 0.5):
        got = _host.select_greedy(ep, preds, alpha, 5, _host.UPDATE_EP, nthreads=4)
        assert got == _scan(ep, preds, alpha, 5, _host.UPDATE_EP)


def test_greedy_runs_out_of_candidates():
    ep = np.array([[5.0, 5.0]])
    preds = np.array([[1.0, 1.0], [6.0, 6.0]])
    assert _host.select_greedy(ep, preds, 0.0, 5, _host.STAIRCASE) == [1, 0]
    assert _host.select_greedy(ep, np.zeros((0, 2)), 0.0, 3, _host.STAIRCASE) == []


# ---------------------------------------------------------------- Pareto primitives
@pytest.mark.parametrize('K', [1, 2, 3])
def test_hypervolume_matches_oracle(K):
    rng = np.random.RandomState(K)
    for n in (0, 1, 2, 5, 30, 120):
        x = rng.rand(n, K) * 50 - 1
        x[::5] = np.round(x[::5])  # ties in every coordinate
        assert _host.hypervolume(x) == ref_pareto.compute_hypervolume(x)


@pytest.mark.parametrize('K', [2, 3, 4])
def test_ep_mask_matches_get_ep_indices(K):
    rng = np.random.RandomState(10 + K)
    x = np.round(rng.rand(300, K) * 20 - 1, 1)  # many ties and duplicates
    keep = _host.ep_mask(x)
    assert sorted(np.nonzero(keep)[0].tolist()) == sorted(int(i) for i in ref_pareto.get_ep_indices(x))
