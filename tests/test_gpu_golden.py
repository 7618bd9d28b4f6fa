"""Device kernels (through the C ABI) against the committed golden vectors only: no oracle at run time.

Tolerances: fp32 device arithmetic vs fp64 golden values, stated per check (north-star bar: scalarised
returns within 1e-5 relative; masks bit-exact).
"""
import numpy as np
import pytest
import torch

from pgmorl_amd import envspec
from pgmorl_amd.runtime import TaskBatch

from .golden_io import RMS, load, state_dict

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol, what):
    a = np.asarray(a.cpu() if isinstance(a, torch.Tensor) else a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, f'{what}: shape {a.shape} != {b.shape}'
    bad = np.abs(a - b) > atol + rtol * np.abs(b)
    assert not bad.any(), f'{what}: {bad.sum()}/{bad.size} off, max abs err {np.abs(a - b).max():.3e}'


def _kernels_batch(g, **kw):
    P, T, N = (int(x) for x in g['dims'][:3])
    tb = TaskBatch('MO-Walker2d-v2', P, num_processes=N, num_steps=T, **kw)
    for p in range(P):
        tb.set_task(p, state_dict(g, f'pol{p}'))
    return tb


def test_golden_act(gpu):
    g = load('kernels')
    tb = _kernels_batch(g)
    v, a, lp = tb.act(torch.from_numpy(g['act/obs']).to(gpu), torch.from_numpy(g['act/noise']).to(gpu))
    _, am, _ = tb.act(torch.from_numpy(g['act/obs']).to(gpu), deterministic=True)
    for p in range(tb.P):
        _close(v[p], g[f'act/value{p}'], 2e-5, 1e-5, 'value')
        _close(a[p], g[f'act/action{p}'], 2e-5, 1e-5, 'action')
        _close(lp[p], g[f'act/logp{p}'], 5e-5, 1e-5, 'logp')
        _close(am[p], g[f'act/mean{p}'], 2e-5, 1e-5, 'deterministic action')


@pytest.mark.parametrize('use_gae', [0, 1])
@pytest.mark.parametrize('proper', [0, 1])
def test_golden_gae(gpu, use_gae, proper):
    g = load('kernels')
    tb = _kernels_batch(g, use_gae=bool(use_gae), use_proper_time_limits=bool(proper), gamma=0.99, gae_lambda=0.95)
    for dst, k in ((tb.rewards, 'rewards'), (tb.values, 'values'), (tb.masks, 'masks'), (tb.bad_masks, 'bad_masks')):
        dst.copy_(torch.from_numpy(g['gae/' + k]))
    tb.gae()
    T = tb.T
    _close(tb.returns[:, :T], g[f'gae/returns_g{use_gae}_p{proper}'][:, :T], 1e-5, 1e-5, 'returns')


@pytest.mark.parametrize('obj_rms', [True, False])
def test_golden_adv(gpu, obj_rms):
    g = load('kernels')
    tb = _kernels_batch(g, obj_rms=obj_rms)
    tb.returns.copy_(torch.from_numpy(g['adv/returns']))
    tb.values.copy_(torch.from_numpy(g['adv/values']))
    tb.weights.copy_(torch.from_numpy(g['adv/weights']))
    tb.obj_var.copy_(torch.from_numpy(g['adv/obj_var']))
    tb.adv_normalize()
    _close(tb.adv, g['adv/adv' if obj_rms else 'adv/adv_noobjrms'], 1e-5, 1e-5, 'advantages')


@pytest.mark.parametrize('kernel', ['mfma', 'mfma-tower', 'mfma-joint', 'valu'])
def test_golden_ppo_update(gpu, kernel, monkeypatch):
    monkeypatch.setenv('PGM_UPDATE_KERNEL', kernel.split('-')[0])
    monkeypatch.setenv('PGM_UPDATE_SPLIT', {'mfma': '2', 'mfma-tower': '1', 'mfma-joint': '0'}.get(kernel, '2'))
    g = load('kernels')
    E = g['ppo/perms'].shape[0]
    tb = _kernels_batch(g, ppo_epoch=E, num_mini_batch=4)
    for dst, k in ((tb.obs, 'obs'), (tb.actions, 'actions'), (tb.logp, 'logp'), (tb.values, 'values'),
                   (tb.returns, 'returns'), (tb.adv, 'adv')):
        dst.copy_(torch.from_numpy(g['ppo/' + k]))
    tb.lr.fill_(float(g['ppo/lr']))
    tb.ppo_update(g['ppo/perms'])
    assert int(tb.update_ws[2 * tb.P]) == 0
    lay = tb.layout
    for p in range(tb.P):
        _close(tb.params[p], lay.flatten(state_dict(g, f'ppo/after{p}'), np.float64), 2e-6, 1e-5, 'params')
        _close(tb.adam_m[p], lay.flatten(state_dict(g, f'ppo/exp_avg{p}'), np.float64), 1e-7, 1e-3, 'exp_avg')
        _close(tb.adam_v[p], lay.flatten(state_dict(g, f'ppo/exp_avg_sq{p}'), np.float64), 1e-10, 1e-3,
               'exp_avg_sq')
        _close(tb.stats[p], g[f'ppo/stats{p}'], 1e-5, 1e-4, 'loss stats')


def test_golden_eval(gpu):
    g = load('kernels')
    tb = _kernels_batch(g, eval_num=1, raw=True)
    for p in range(tb.P):
        tb.set_env_params(p, {'ob_rms': RMS(g[f'eval/ob_mean{p}'], g[f'eval/ob_var{p}'], g[f'eval/ob_count{p}'])})
    objs = tb.evaluate()
    for p in range(tb.P):
        _close(objs[p], g[f'eval/objs{p}'], 1e-4, 1e-5, 'evaluation objs')


def test_golden_mopg_two_iterations(gpu):
    """Two MOPG iterations of one Hopper-v2 task with the reference's RNG draws."""
    g = load('mopg')
    T, N, E, M, iters = (int(x) for x in g['dims'])
    tb = TaskBatch('MO-Hopper-v2', 1, num_processes=N, num_steps=T, ppo_epoch=E, num_mini_batch=M)
    tb.set_task(0, state_dict(g, 'init'), None, None, g['weights'])
    tb.env_reset()
    total = int(g['num_env_steps']) // T // N
    lay = tb.layout
    for j in range(iters):
        lr = 3e-4 * (1.0 - j / float(total))
        tb.iteration(j, lr, noise=torch.from_numpy(g[f'it{j}/noise']).to(gpu), perms=g[f'it{j}/perms'], carry=j > 0)
        _close(tb.obs[0], g[f'it{j}/obs'], 5e-5, 1e-4, f'obs it{j}')
        _close(tb.actions[0], g[f'it{j}/actions'], 5e-5, 1e-4, f'actions it{j}')
        np.testing.assert_array_equal(tb.masks[0].cpu().numpy(), g[f'it{j}/masks'])
        np.testing.assert_array_equal(tb.bad_masks[0].cpu().numpy(), g[f'it{j}/bad_masks'])
        _close(tb.rewards[0], g[f'it{j}/rewards'], 5e-5, 1e-4, f'rewards it{j}')
        _close(tb.returns[0, :T], g[f'it{j}/returns'][:T], 1e-4, 1e-4, f'returns it{j}')
        _close(tb.obj_var[0], g[f'it{j}/obj_var_end'], 0, 1e-6, f'obj_rms.var it{j}')
        _close(tb.ob_mean[0], g[f'it{j}/ob_mean'], 1e-7, 1e-6, f'ob_rms.mean it{j}')
        _close(tb.params[0], lay.flatten(state_dict(g, f'it{j}/params'), np.float64), 2e-5, 1e-4, f'params it{j}')
        _close(tb.objs[0], g[f'it{j}/objs'], 1e-3, 1e-4, f'eval objs it{j}')
