"""Pinning the CPU oracle: the reference's own known-answer test pattern, closed forms of the
third-party arithmetic it relies on (torch Normal, Adam, clip_grad_norm_, randperm/normal draws),
and hand-computed Pareto / hypervolume cases."""
import numpy as np
import pytest
import torch

from oracle import pareto, ppo as oppo
from oracle.policy import make_policy
from oracle.vecenv import RunningMeanStd, SynthEnv, VecNormalizedSynth
from pgmorl_amd import envspec


# ---------------------------------------------------------------- RunningMeanStd
def test_runningmeanstd_reference_kat():
    """externals/baselines/baselines/common/running_mean_std.py:85-100 (test_runningmeanstd)."""
    rng = np.random.RandomState(0)
    for (x1, x2, x3) in [(rng.randn(3), rng.randn(4), rng.randn(5)),
                         (rng.randn(3, 2), rng.randn(4, 2), rng.randn(5, 2))]:
        rms = RunningMeanStd(epsilon=0.0, shape=x1.shape[1:])
        x = np.concatenate([x1, x2, x3], axis=0)
        rms.update(x1)
        rms.update(x2)
        rms.update(x3)
        np.testing.assert_allclose([x.mean(axis=0), x.var(axis=0)], [rms.mean, rms.var])


def test_obj_rms_scalar_shape_broadcasts_to_K():
    """vec_normalize.py:21,45: obj_rms is created with shape () and becomes (K,) on first update."""
    r = RunningMeanStd(shape=())
    r.update(np.array([[1.0, 2.0], [3.0, 5.0]]))
    assert r.mean.shape == (2,)
    want_mean = (np.array([2.0, 3.5]) * 2) / (2 + 1e-4)
    np.testing.assert_allclose(r.mean, want_mean)


# ---------------------------------------------------------------- policy / distributions
def test_policy_init_matches_reference_construction_order():
    """Initial params depend on the RNG draws of every Linear default init + orthogonal re-init,
    including the discarded 1-output critic_linear (model.py:233,254)."""
    torch.manual_seed(0)
    p = make_policy(17, 6, 2)
    torch.manual_seed(0)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        import torch.nn as nn
        mods = []
        for _ in range(2):  # actor, critic towers
            for fan_in in (17, 64):
                lin = nn.Linear(fan_in, 64)
                nn.init.orthogonal_(lin.weight.data, gain=np.sqrt(2))
                mods.append(lin)
        h1 = nn.Linear(64, 1)
        nn.init.orthogonal_(h1.weight.data, gain=np.sqrt(2))
        hk = nn.Linear(64, 2)
        nn.init.orthogonal_(hk.weight.data, gain=np.sqrt(2))
        fm = nn.Linear(64, 6)
        nn.init.orthogonal_(fm.weight.data, gain=1.0)
    finally:
        torch.set_default_dtype(prev)
    assert torch.equal(p.base.actor[0].weight, mods[0].weight)
    assert torch.equal(p.base.critic[2].weight, mods[3].weight)
    assert torch.equal(p.base.critic_linear.weight, hk.weight)
    assert torch.equal(p.dist.fc_mean.weight, fm.weight)
    assert torch.all(p.base.actor[0].bias == 0) and torch.all(p.dist.logstd._bias == 0)


def test_normal_logprob_entropy_closed_form():
    torch.manual_seed(1)
    p = make_policy(11, 3, 2)
    with torch.no_grad():
        p.dist.logstd._bias.copy_(torch.tensor([[0.1], [-0.3], [0.2]]))
    x = torch.randn(5, 11, dtype=torch.float64)
    a = torch.randn(5, 3, dtype=torch.float64)
    v, lp, ent = p.evaluate_actions(x, a)
    mu = p.dist.fc_mean(p.base.actor(x))
    ls = p.dist.logstd._bias[:, 0]
    want = (-(a - mu) ** 2 / (2 * torch.exp(2 * ls)) - ls - 0.5 * np.log(2 * np.pi)).sum(-1, keepdim=True)
    torch.testing.assert_close(lp, want)
    torch.testing.assert_close(ent, (0.5 + 0.5 * np.log(2 * np.pi) + ls).sum())


def test_sample_equals_explicit_noise():
    """Normal.sample == torch.normal(mean, std) == z*std + mean with z drawn by torch.normal(0, 1):
    the extracted noise reproduces the reference's own RNG draws bit for bit."""
    torch.manual_seed(2)
    p = make_policy(17, 6, 2)
    x = torch.randn(4, 17, dtype=torch.float64)
    torch.manual_seed(9)
    _, a_native, lp_native = p.act(x)
    torch.manual_seed(9)
    z = torch.normal(torch.zeros(4, 6, dtype=torch.float64), torch.ones(4, 6, dtype=torch.float64))
    _, a_noise, lp_noise = p.act(x, noise=z)
    assert torch.equal(a_native, a_noise) and torch.equal(lp_native, lp_noise)


def test_adam_and_clip_closed_form():
    """torch Adam (lerp m, v, bias-corrected step, eps outside sqrt) + clip_grad_norm_."""
    w = torch.nn.Parameter(torch.tensor([1.0, -2.0, 3.0], dtype=torch.float64))
    opt = torch.optim.Adam([w], lr=0.1, eps=1e-5)
    m = np.zeros(3)
    v = np.zeros(3)
    x = w.detach().numpy().copy()
    for step in range(1, 4):
        opt.zero_grad()
        (w * torch.tensor([3.0, 4.0, 0.5], dtype=torch.float64) * step).sum().backward()
        total = torch.nn.utils.clip_grad_norm_([w], 0.5)
        g = np.array([3.0, 4.0, 0.5]) * step
        coef = min(0.5 / (np.linalg.norm(g) + 1e-6), 1.0)
        assert float(total) == pytest.approx(np.linalg.norm(g))
        g = g * coef
        opt.step()
        m = m + 0.1 * (g - m)
        v = 0.999 * v + 0.001 * g * g
        x = x - (0.1 / (1 - 0.9 ** step)) * m / (np.sqrt(v) / np.sqrt(1 - 0.999 ** step) + 1e-5)
        np.testing.assert_allclose(w.detach().numpy(), x, rtol=1e-12)


def test_update_uses_one_randperm_per_epoch():
    """SubsetRandomSampler draws torch.randperm(T*N) once per epoch (the extracted perms)."""
    torch.manual_seed(4)
    want = [torch.randperm(64) for _ in range(3)]
    torch.manual_seed(4)
    got = oppo.randperms(3, 64)
    assert all(torch.equal(a, b) for a, b in zip(want, got))


# ---------------------------------------------------------------- returns
def test_gae_closed_form_small():
    T, N, K = 3, 1, 1
    r = torch.tensor([[[1.0]], [[2.0]], [[3.0]]], dtype=torch.float64)
    v = torch.tensor([[[0.5]], [[0.25]], [[0.125]], [[1.0]]], dtype=torch.float64)
    m = torch.ones(T + 1, N, 1, dtype=torch.float64)
    b = torch.ones(T + 1, N, 1, dtype=torch.float64)
    m[2] = 0.0  # episode ends after step 1 (true terminal)
    ret = torch.zeros(T + 1, N, K, dtype=torch.float64)
    g, lam = 0.9, 0.8
    oppo.compute_returns_inplace(r, v.clone(), m, b, ret, v[-1], True, g, lam, True)
    d2 = 3.0 + g * 1.0 * 1 - 0.125
    d1 = 2.0 + g * 0.125 * 0 - 0.25
    d0 = 1.0 + g * 0.25 * 1 - 0.5
    a2 = d2
    a1 = d1
    a0 = d0 + g * lam * a1
    np.testing.assert_allclose(ret[:3, 0, 0].numpy(), [a0 + 0.5, a1 + 0.25, a2 + 0.125])


def test_advantage_uses_unbiased_std():
    R = torch.tensor([[[1.0, 0.0]], [[3.0, 0.0]], [[2.0, 0.0]], [[0.0, 0.0]]], dtype=torch.float64)
    V = torch.zeros_like(R)
    adv = oppo.scalarized_normalized_advantages(R, V, [1.0, 0.0], None)
    x = np.array([1.0, 3.0, 2.0])
    np.testing.assert_allclose(adv[:, 0].numpy(), (x - x.mean()) / (x.std(ddof=1) + 1e-5))


# ---------------------------------------------------------------- synthetic env stack
def test_synth_env_time_limit_and_autoreset():
    spec = envspec.make_spec('MO-Hopper-v2')
    s0 = envspec.reset_table(spec['obs_dim'], 0, 2)
    venv = VecNormalizedSynth(spec, s0, 0.995)
    venv.reset()
    for t in range(1, 501):
        obs, dones, infos = venv.step(np.zeros((2, 3)))
        if t < 500:
            assert not dones.any()
        else:
            assert dones.all() and all('bad_transition' in i for i in infos)
    assert all(e.elapsed == 0 for e in venv.envs)
    np.testing.assert_array_equal(venv.envs[0].s, s0[0])
    assert np.all(venv.obj == 0)


def test_env_objective_form():
    spec = envspec.make_spec('MO-Walker2d-v2')
    e = SynthEnv(spec, envspec.reset_state(17, 0))
    e.reset()
    a = np.array([2.0, -0.5, 0.1, 0.0, 0.3, -3.0])
    s_prev = e.s.copy()
    _, _, _, info = e.step(a)
    ac = np.clip(a, -1, 1)
    s = np.tanh(spec['d'] * s_prev + spec['U'] @ ac + spec['c'])
    np.testing.assert_allclose(info['obj'], [spec['V'][0] @ s + 1.0, 5.0 - np.sum(ac ** 2)])


# ---------------------------------------------------------------- Pareto archive / HV / weights
def test_get_ep_indices_drops_dominated_negative_keeps_duplicates():
    objs = np.array([[1.0, 5.0], [2.0, 4.0], [1.5, 3.0], [3.0, -0.1], [2.0, 4.0], [0.5, 5.0]])
    idx = pareto.get_ep_indices(objs)
    assert sorted(idx) == [0, 1, 4]
    assert [objs[i][0] for i in idx] == sorted(objs[i][0] for i in idx)


def test_hypervolume_2d_and_3d_by_hand():
    assert pareto.compute_hypervolume([[1.0, 3.0], [2.0, 2.0], [3.0, 1.0]]) == 6.0
    assert pareto.compute_hypervolume([[2.0, 2.0, 2.0]]) == 8.0
    assert pareto.compute_hypervolume([[2.0, 1.0, 1.0], [1.0, 2.0, 1.0], [1.0, 1.0, 2.0]]) == 4.0
    hv, sp = pareto.hv_sparsity_2d(np.array([[1.0, 3.0], [2.0, 2.0], [3.0, 1.0]]))
    assert hv == 6.0 and sp == pytest.approx(2.0)


def test_weight_grid_dfs_counts_and_quirks():
    for delta, n in ((0.25, 5), (1 / 39, 40), (1 / 159, 160)):
        wb = []
        pareto.generate_weights_batch_dfs(0, 2, 0.0, 1.0, delta, [], wb)
        assert len(wb) == n
    wb = []
    pareto.generate_weights_batch_dfs(0, 3, 0.0, 1.0, 1 / 19, [], wb)
    assert len(wb) == 210
    wb = []
    pareto.generate_weights_batch_dfs(0, 2, 0.0, 1.0, 0.1, [], wb)
    assert wb[-1][0] > 1.0 - 1e-9 and abs(wb[-1][1]) < 1e-9  # accumulated w += delta quirk kept
