"""The update launch the bench times, whole: E = 10 epochs x M = 32 minibatches = 320 Adam steps per task in ONE
pgm_ppo_update launch (a2c_ppo_acktr/algo/ppo.py:58-115, storage.py:118-154: the perms of all ten epochs, every parity
slot of the hand-offs cycled 160 times, the ragged parts' dummy tiles re-zeroed every step), at the per-GPU loads of
config 0 (Hopper-v2 P = 5, N = 1: 64-row minibatches, NS 4, R 1), config 1 (Walker P = 40: NS 6, R 3/3/3/3/2/2, two
workgroups per CU), config 2 (HalfCheetah P = 20: NS 8, R 2, two per CU), config 3 (Hopper-v3 P = 27: three
objectives, a partial last group of 8 tasks) and config 4 (Humanoid P = 20, N = 8: the wide update, NS 4, 512-row
minibatches, the private k-quad layer-1 copies carried over all 320 steps and written back once, the next minibatch's
rows prefetched across epoch ends).
Every task against the oracle.

Tolerance (drift-aware, not a loosened constant): over 320 Adam steps fp32 arithmetic drifts from the fp64 reference;
the oracle's own fp32 arm (the same restatement with the policy, losses, backward and Adam in fp32, oracle/mopg.py NET)
measures that drift per task, d32 = max |o32 - o64| (~1e-6 at Walker dims).  The device must stay within
DRIFT_FACTOR x d32 + 2e-6 of a reference trajectory in every parameter (the short launches' bound is 2e-6 + 1e-5 rel),
its Adam moments likewise, and its mean loss statistics within 1e-4 relative.

The reference trajectory is the fp64 oracle -- or, for a task whose update is SENSITIVE, one of the trajectories fp32
rounding reaches: a few tasks in 60 hit a discontinuity of the loss (a sample's ratio at the clip boundary, a
torch.min/max tie) within rounding at some Adam step, after which the trajectory jumps by ~1e-3 (HalfCheetah P = 20
task 15 at step 147: the fp32 oracle started from parameters 1 ulp away from the test's ends exactly where the device
does, 9.3667e-4 from the fp64 one).  For a task the device does not match within the band of the fp64 oracle or its
fp32 arm, the fp32 arm is re-run from up to MAX_PERTURBED initial parameter sets each 1 ulp (2^-23 relative, random
signs) away from the test's, and the device must match one of them within the same band.  Every such task is listed
in gpurun_out/long_update_<env>.json with the arm that matched (and the counts must stay small).

Humanoid is CHAOTIC at this horizon: its 376-input policy on 16384 rows x 320 steps puts a flip in most trajectories
(the fp32 oracle itself ends 1e-3 - 6e-3 off the fp64 one in about half the tasks, while the other half agree to
1e-6), so a 1-ulp arm rarely replays the device's exact flips.  There the device must match a trajectory within the
rounding band (measured on the unflipped fp32 arms only) in at least half the tasks, end off every trajectory tried
in no more tasks than the fp32 oracle ends off the fp64 one, and only by a jump no larger than twice the oracle's own
largest flip.  A defect of the launch itself (layer-1 copies, the cross-minibatch prefetch, a flag slot) would move
every task, including the unflipped half."""
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
MAX_PERTURBED = 8     # 1-ulp fp32 arms tried for a task off both unperturbed bands
MAX_SENSITIVE = 0.25  # at most this share of the tasks may need a perturbed arm
FLIP = 1e-4           # |o32 - o64| above this is a flip of the loss (~1e-3), not rounding drift (~1e-6)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle_arm(pol, args, data, p, perms, E, M, T, N, spec, lr, dtype, pert_seed=None):
    obs, actions, logp, values, returns, adv = data
    pol = copy.deepcopy(pol)
    if pert_seed is not None:  # every parameter 1 ulp (fp32) up or down
        g = torch.Generator().manual_seed(pert_seed)
        with torch.no_grad():
            for q in pol.parameters():
                q.mul_(1 + 2.0 ** -23 * torch.randn(q.shape, generator=g, dtype=torch.float64).sign())
    pol = pol.to(dtype)
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


@pytest.mark.parametrize('env,P,N,variant,chaotic', [
    ('MO-Walker2d-v2', 40, 4, 'ppo_update_fs_kernel (NS=6, R=3, 2 per CU)', False),
    ('MO-HalfCheetah-v2', 20, 4, 'ppo_update_fs_kernel (NS=8, R=2, 2 per CU)', False),
    ('MO-Hopper-v3', 27, 4, 'ppo_update_fs_kernel (NS=8, R=2, 2 per CU)', False),
    ('MO-Hopper-v2', 5, 1, 'ppo_update_fs_kernel (NS=4, R=1)', False),
    ('MO-Humanoid-v2', 20, 8, 'ppo_update_wide_kernel (NS=4)', True)])
def test_full_production_update_launch(gpu, env, P, N, variant, chaotic):
    T, E, M, lr = 2048, 10, 32, 3e-4
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

    def dist(pp, mm, vv, st, pol, ag, stt):
        r = torch.from_numpy(L.flatten(pol.state_dict(), dtype=np.float64))
        m_, v_, _ = L.adam_from_optimizer_state(ag.optimizer.state_dict()['state'])
        m_, v_ = torch.as_tensor(m_, dtype=torch.float64), torch.as_tensor(v_, dtype=torch.float64)
        return ((pp - r).abs().max().item(), (mm - m_).abs().max().item(),
                ((vv - v_).abs() / (v_.abs() + 1e-12)).max().item(),
                (np.abs(st - stt) / (np.abs(stt) + 1e-6)).max().item())

    def as_dev(pol, ag, st):
        m_, v_, _ = L.adam_from_optimizer_state(ag.optimizer.state_dict()['state'])
        return (torch.from_numpy(L.flatten(pol.state_dict(), dtype=np.float64)), torch.as_tensor(m_, dtype=torch.float64),
                torch.as_tensor(v_, dtype=torch.float64), st)

    # the fp32 rounding drift of an unflipped task: the median of |o32 - o64| over the tasks whose fp32 arm did not
    # flip (a flipped task's distance is ~1e3 x larger and must not widen the band)
    d32s = [dist(*as_dev(pol32, ag32, st32), pol64, ag64, st64) for (pol64, ag64, st64), (pol32, ag32, st32) in arms]
    calm = [d for d in d32s if d[0] < FLIP]
    assert len(calm) >= P // 4, (env, 'too few unflipped fp32 arms to measure the rounding drift', len(calm))
    drift = [float(np.median([d[i] for d in calm])) for i in range(4)]
    band = (DRIFT_FACTOR * drift[0] + 2e-6, DRIFT_FACTOR * drift[1] + 1e-7, DRIFT_FACTOR * drift[2] + 1e-3,
            max(1e-4, DRIFT_FACTOR * drift[3]))

    def within(d):
        return all(x <= b for x, b in zip(d, band))

    def dev(p):
        return params[p], am[p], av[p], stats[p].numpy()
    first = []
    for p, ((pol64, ag64, st64), (pol32, ag32, st32)) in enumerate(arms):
        _, _, step = L.adam_from_optimizer_state(ag64.optimizer.state_dict()['state'])
        assert int(steps[p]) == step == E * M
        d_dev64, d_dev32 = dist(*dev(p), pol64, ag64, st64), dist(*dev(p), pol32, ag32, st32)
        first.append(('fp64', d_dev64) if within(d_dev64) else ('fp32', d_dev32) if within(d_dev32) else (None, d_dev64))
    # tasks off both unperturbed bands: the 1-ulp fp32 arms, all run at once on the thread pool
    off = [p for p in range(P) if first[p][0] is None]
    torch.set_num_threads(1)
    try:
        with ThreadPoolExecutor(max_workers=16) as ex:
            pert = dict(zip([(p, ps) for p in off for ps in range(MAX_PERTURBED)],
                            ex.map(lambda a: _oracle_arm(pols[a[0]], args, data, a[0], perms, E, M, T, N, spec, lr,
                                                         torch.float32, pert_seed=a[1]),
                                   [(p, ps) for p in off for ps in range(MAX_PERTURBED)])))
    finally:
        torch.set_num_threads(nthr)
    report = []
    for p in range(P):
        d32, (matched, d_best), d_dev64 = d32s[p], first[p], dist(*dev(p), *arms[p][0])
        if matched is None:
            for ps in range(MAX_PERTURBED):
                d = dist(*dev(p), *pert[(p, ps)])
                if within(d):
                    matched, d_best = f'fp32, 1 ulp (seed {ps})', d
                    break
        report.append({'task': p, 'matched': matched, 'param_d32': d32[0], 'param_ddev': d_dev64[0],
                       'param_d_matched': d_best[0], 'adam_m_d32': d32[1], 'adam_m_ddev': d_dev64[1],
                       'adam_v_rel_d32': d32[2], 'adam_v_rel_ddev': d_dev64[2], 'stats_rel': d_dev64[3],
                       'stats_rel_32': d32[3]})
    out = os.path.join(ROOT, 'gpurun_out')
    os.makedirs(out, exist_ok=True)
    summ = {'env': env, 'P': P, 'variant': variant, 'adam_steps': E * M, 'device_s': dev_s, 'oracle_s': oracle_s,
            'drift_median': drift, 'band': band,
            'max_param_ddev': max(r['param_ddev'] for r in report), 'max_param_d32': max(r['param_d32'] for r in report),
            'max_param_d_matched': max(r['param_d_matched'] for r in report),
            'matched': {k: sum(r['matched'] == k for r in report) for k in {r['matched'] for r in report}},
            'sensitive_tasks': [r['task'] for r in report if r['matched'] not in ('fp64',)],
            'fp32_arm_flips': [p for p in range(P) if d32s[p][0] >= FLIP], 'tasks': report}
    with open(os.path.join(out, f'long_update_{env}.json'), 'w') as f:
        json.dump(summ, f, indent=1)
    print(json.dumps({k: v for k, v in summ.items() if k != 'tasks'}))
    unmatched = [r for r in report if r['matched'] is None]
    if not chaotic:
        assert not unmatched, (env, unmatched)
        perturbed = [r['task'] for r in report if r['matched'].startswith('fp32, 1 ulp')]
        assert len(perturbed) <= MAX_SENSITIVE * P, (env, perturbed)
    else:
        # the fp32 oracle itself ends off the fp64 trajectory in n_flip32 tasks: the device may end off every
        # trajectory tried in no more tasks than that, only by a jump of the oracle's own flip size, and at least
        # half the tasks must match a trajectory within the rounding band
        n_flip32 = sum(d[0] >= FLIP for d in d32s)
        assert len(unmatched) <= n_flip32, (env, len(unmatched), n_flip32)
        assert len(unmatched) <= P // 2, (env, [r['task'] for r in unmatched])
        big = max(d[0] for d in d32s)
        assert all(r['param_ddev'] <= 2 * big for r in unmatched), (env, big, unmatched)
