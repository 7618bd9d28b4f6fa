"""The committed golden vectors (tests/golden/) against the spec generator and the CPU oracle.

Pins (i) the SynthMO constants bit-exactly, and (ii) the oracle's outputs, so that neither can drift
silently under the device parity tests (tests/test_gpu_golden.py), which read only these fixtures.
"""
import numpy as np
import pytest
import torch

from oracle import ppo as oppo
from oracle.mopg import evaluation, mopg_worker, OracleSample
from oracle.policy import make_policy
from oracle.vecenv import RunningMeanStd
from pgmorl_amd import envspec

from .golden.make_golden import ENV_KEYS, _args, host_draws
from .golden_io import load, state_dict


def _close(a, b, tol, what):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape, f'{what}: shape {a.shape} != {b.shape}'
    err = np.abs(a - b) / (1.0 + np.abs(b))
    assert err.max(initial=0.0) <= tol, f'{what}: max rel err {err.max():.3e}'


@pytest.mark.parametrize('env', envspec.env_names())
def test_synth_env_constants_pinned(env):
    g = load('synth_env')
    s = envspec.make_spec(env)
    for k in ENV_KEYS:
        np.testing.assert_array_equal(s[k], g[f'{env}/{k}'], err_msg=k)
    np.testing.assert_array_equal([s['obs_dim'], s['act_dim'], s['obj_num'], s['max_episode_steps']],
                                  g[f'{env}/dims'])
    np.testing.assert_array_equal(envspec.reset_table(s['obs_dim'], 0, 8), g[f'{env}/s0'])


def _policy(g, prefix, spec):
    pol = make_policy(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
    pol.load_state_dict(state_dict(g, prefix))
    return pol


def test_oracle_matches_golden_kernels():
    g = load('kernels')
    P, T, N, O, A, K = (int(x) for x in g['dims'])
    spec = envspec.make_spec('MO-Walker2d-v2')
    pols = [_policy(g, f'pol{p}', spec) for p in range(P)]
    for p, pol in enumerate(pols):
        with torch.no_grad():
            v, a, lp = pol.act(torch.from_numpy(g['act/obs'][p]).double(),
                               noise=torch.from_numpy(g['act/noise']).double())
        _close(v, g[f'act/value{p}'], 1e-12, 'act value')
        _close(a, g[f'act/action{p}'], 1e-12, 'act action')
        _close(lp[:, 0], g[f'act/logp{p}'], 1e-12, 'act logp')
    for ug in (0, 1):
        for pr in (0, 1):
            for p in range(P):
                ret = torch.zeros(T + 1, N, K, dtype=torch.float64)
                v = torch.from_numpy(g['gae/values'][p]).double()
                oppo.compute_returns_inplace(torch.from_numpy(g['gae/rewards'][p]).double(), v.clone(),
                                             torch.from_numpy(g['gae/masks'][p]).double().unsqueeze(-1),
                                             torch.from_numpy(g['gae/bad_masks'][p]).double().unsqueeze(-1),
                                             ret, v[-1], bool(ug), 0.99, 0.95, bool(pr))
                _close(ret, g[f'gae/returns_g{ug}_p{pr}'][p], 1e-12, 'gae')
    for p in range(P):
        adv = oppo.scalarized_normalized_advantages(torch.from_numpy(g['adv/returns'][p]).double(),
                                                    torch.from_numpy(g['adv/values'][p]).double(),
                                                    g['adv/weights'][p], g['adv/obj_var'][p])
        _close(adv, g['adv/adv'][p], 1e-12, 'adv')
    E, M = g['ppo/perms'].shape[0], 4
    for p in range(P):
        pol = _policy(g, f'pol{p}', spec)
        agent = oppo.PPO(pol, 0.2, E, M, 0.5, 0.0, lr=float(g['ppo/lr']), eps=1e-5, max_grad_norm=0.5)
        ro = oppo.RolloutStorage(T, N, O, A, K)
        ro.obs.copy_(torch.from_numpy(g['ppo/obs'][p]).double())
        ro.actions.copy_(torch.from_numpy(g['ppo/actions'][p]).double())
        ro.action_log_probs.copy_(torch.from_numpy(g['ppo/logp'][p]).double().unsqueeze(-1))
        ro.value_preds.copy_(torch.from_numpy(g['ppo/values'][p]).double())
        ro.returns.copy_(torch.from_numpy(g['ppo/returns'][p]).double())
        for e in range(E):
            for mbt in ro.minibatches(torch.from_numpy(g['ppo/adv'][p]).double(), M,
                                      torch.from_numpy(g['ppo/perms'][e]).long()):
                agent.minibatch_step(*mbt)
        want = state_dict(g, f'ppo/after{p}')
        for k, v in pol.state_dict().items():
            _close(v, want[k], 1e-10, f'ppo {k}')
    s0_eval = envspec.reset_table(O, 0, 1)
    for p, pol in enumerate(pols):
        r = RunningMeanStd(shape=(O,))
        r.mean, r.var, r.count = g[f'eval/ob_mean{p}'], g[f'eval/ob_var{p}'], float(g[f'eval/ob_count{p}'])
        _close(evaluation(_args('MO-Walker2d-v2'), spec, s0_eval, pol, r), g[f'eval/objs{p}'], 1e-10, 'eval')


def test_oracle_matches_golden_mopg():
    g = load('mopg')
    T, N, E, M, iters = (int(x) for x in g['dims'])
    env = 'MO-Hopper-v2'
    spec = envspec.make_spec(env)
    args = _args(env, num_steps=T, num_processes=N, ppo_epoch=E, num_mini_batch=M,
                 num_env_steps=int(g['num_env_steps']))
    pol = _policy(g, 'init', spec)
    agent = oppo.PPO(pol, 0.2, E, M, 0.5, 0.0, lr=3e-4, eps=1e-5, max_grad_norm=0.5)
    sample = OracleSample({'ob_rms': RunningMeanStd(shape=(spec['obs_dim'],)), 'ret_rms': RunningMeanStd(shape=()),
                           'obj_rms': RunningMeanStd(shape=())}, pol, agent, optgraph_id=-1)
    fn = host_draws(T, N, spec['act_dim'], E)
    for j in range(iters):  # the committed draws are the reference's torch draws of iteration j
        noise, perms = fn(j)
        np.testing.assert_array_equal(noise.float().numpy(), g[f'it{j}/noise'])
        np.testing.assert_array_equal(torch.stack(perms).numpy(), g[f'it{j}/perms'])
    offs = mopg_worker(args, spec, envspec.reset_table(spec['obs_dim'], 0, N), envspec.reset_table(spec['obs_dim'], 0, 1),
                       sample, g['weights'], 0, iters,
                       noise_fn=lambda j: (fn(j)[0].float().double(), fn(j)[1]))
    for j, off in enumerate(offs):
        want = state_dict(g, f'it{j}/params')
        for k, v in off.actor_critic.state_dict().items():
            _close(v, want[k], 1e-9, f'iter {j} {k}')
        _close(off.objs, g[f'it{j}/objs'], 1e-9, f'iter {j} objs')
