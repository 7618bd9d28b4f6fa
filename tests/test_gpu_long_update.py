"""The update launch the bench times, whole: E = 10 epochs x M = 32 minibatches = 320 Adam steps per task in ONE
pgm_ppo_update launch (a2c_ppo_acktr/algo/ppo.py:58-115, storage.py:118-154: the perms of all ten epochs, every parity
slot of the hand-offs cycled 160 times, the ragged parts' dummy tiles re-zeroed every step), at the per-GPU loads of
config 1 (Walker P = 40: NS 6, R 3/3/3/3/2/2, two workgroups per CU) and config 2 (HalfCheetah P = 20: NS 8, R 2, two
per CU).  Every task against the oracle.

Tolerance (drift-aware, not a loosened constant): over 320 Adam steps fp32 arithmetic drifts from the fp64 reference;
the oracle's own fp32 arm (the same restatement with the policy, losses, backward and Adam in fp32, oracle/mopg.py NET)
measures that drift per task, d32 = max |o32 - o64| (~1e-6 at Walker dims).  The device must stay within
DRIFT_FACTOR x d32 + 2e-6 of the fp64 oracle in every parameter (the short launches' bound is 2e-6 + 1e-5 rel), its Adam
moments likewise, and its mean loss statistics within 1e-4 relative.  The measured ratios are written to
gpurun_out/long_update_<env>.json."""
import copy
import json
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from oracle import ppo as oppo

from .test_gpu_kernels import _update_setup

pytestmark = pytest.mark.gpu

DRIFT_FACTOR = 8.0
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle_arm(pol, args, data, p, perms, E, M, T, N, spec, lr, dtype):
    obs, actions, logp, values, returns, adv = data
    pol = copy.deepcopy(pol).to(dtype)
    agent = oppo.PPO(pol, args.clip_param, E, M, args.value_loss_coef, args.entropy_coef, lr=lr, eps=1e-5,
                     max_grad_norm=args.max_grad_norm)
    ro = oppo.RolloutStorage(T, N, spec['obs_dim'], spec['act_dim'], spec['obj_num'])
    ro.obs.copy_(torch.from_numpy(obs[p]).double())
    ro.actions.copy_(actions[p].double())
    ro.action_log_probs.copy_(logp[p].double().unsqueeze(-1))
    ro.value_preds.copy_(values[p].double())
    ro.returns.copy_(returns[p].double())
    st = np.zeros(3)
    for e in range(E):
        for mbt in ro.minibatches(adv[p].double(), M, perms[e]):
            if dtype != torch.float64:
                mbt = [x.to(dtype) if torch.is_tensor(x) and x.is_floating_point() else x for x in mbt]
            st += agent.minibatch_step(*mbt)
    return pol.double(), agent, st / (E * M)


@pytest.mark.parametrize('env,P,variant', [('MO-Walker2d-v2', 40, 'ppo_update_fs_kernel (NS=6, R=3, 2 per CU)'),
                                           ('MO-HalfCheetah-v2', 20, 'ppo_update_fs_kernel (NS=8, R=2, 2 per CU)')])
def test_full_production_update_launch(gpu, env, P, variant):
    T, N, E, M, lr = 2048, 4, 10, 32, 3e-4
    args, spec, tb, pols, data, perms = _update_setup(env, P, T, N, E, M, seed=53)
    assert tb.update_variant() == variant  # the launch bench.py times at this load
    tb.lr.fill_(lr)
    torch.cuda.synchronize()
    t0 = time.time()
    tb.ppo_update(torch.stack(perms).numpy())
    tb.check_update()
    dev_s = time.time() - t0
    params, am, av = tb.params.cpu().double(), tb.adam_m.cpu().double(), tb.adam_v.cpu().double()
    steps, stats = tb.adam_step.cpu(), tb.stats.cpu().double()
    L = tb.layout

    def one(p):
        o64 = _oracle_arm(pols[p], args, data, p, perms, E, M, T, N, spec, lr, torch.float64)
        o32 = _oracle_arm(pols[p], args, data, p, perms, E, M, T, N, spec, lr, torch.float32)
        return o64, o32

    nthr = torch.get_num_threads()
    torch.set_num_threads(1)
    t0 = time.time()
    try:
        with ThreadPoolExecutor(max_workers=16) as ex:
            arms = list(ex.map(one, range(P)))
    finally:
        torch.set_num_threads(nthr)
    oracle_s = time.time() - t0
    report = []
    for p, ((pol64, ag64, st64), (pol32, ag32, st32)) in enumerate(arms):
        r64 = torch.from_numpy(L.flatten(pol64.state_dict(), dtype=np.float64))
        r32 = torch.from_numpy(L.flatten(pol32.state_dict(), dtype=np.float64))
        m64, v64, step = L.adam_from_optimizer_state(ag64.optimizer.state_dict()['state'])
        m32, v32, _ = L.adam_from_optimizer_state(ag32.optimizer.state_dict()['state'])
        m64, v64 = torch.as_tensor(m64, dtype=torch.float64), torch.as_tensor(v64, dtype=torch.float64)
        m32, v32 = torch.as_tensor(m32, dtype=torch.float64), torch.as_tensor(v32, dtype=torch.float64)
        assert int(steps[p]) == step == E * M
        d32 = (r32 - r64).abs().max().item()
        ddev = (params[p] - r64).abs().max().item()
        dm32 = (m32 - m64).abs().max().item()
        dmdev = (am[p] - m64).abs().max().item()
        dvdev = ((av[p] - v64).abs() / (v64.abs() + 1e-12)).max().item()
        dv32 = ((v32 - v64).abs() / (v64.abs() + 1e-12)).max().item()
        report.append({'task': p, 'param_d32': d32, 'param_ddev': ddev, 'adam_m_d32': dm32, 'adam_m_ddev': dmdev,
                       'adam_v_rel_d32': dv32, 'adam_v_rel_ddev': dvdev,
                       'stats_rel': (np.abs(stats[p].numpy() - st64) / (np.abs(st64) + 1e-6)).max().item(),
                       'stats_rel_32': (np.abs(st32 - st64) / (np.abs(st64) + 1e-6)).max().item()})
    out = os.path.join(ROOT, 'gpurun_out')
    os.makedirs(out, exist_ok=True)
    summ = {'env': env, 'P': P, 'variant': variant, 'adam_steps': E * M, 'device_s': dev_s, 'oracle_s': oracle_s,
            'max_param_ddev': max(r['param_ddev'] for r in report), 'max_param_d32': max(r['param_d32'] for r in report),
            'max_ratio': max(r['param_ddev'] / max(r['param_d32'], 1e-12) for r in report), 'tasks': report}
    with open(os.path.join(out, f'long_update_{env}.json'), 'w') as f:
        json.dump(summ, f, indent=1)
    print(json.dumps({k: v for k, v in summ.items() if k != 'tasks'}))
    for r in report:
        p = r['task']
        assert r['param_ddev'] <= DRIFT_FACTOR * r['param_d32'] + 2e-6, (env, r)
        assert r['adam_m_ddev'] <= DRIFT_FACTOR * r['adam_m_d32'] + 1e-7, (env, r)
        assert r['adam_v_rel_ddev'] <= DRIFT_FACTOR * r['adam_v_rel_d32'] + 1e-3, (env, r)
        assert r['stats_rel'] <= max(1e-4, DRIFT_FACTOR * r['stats_rel_32']), (env, r, stats[p])
