"""The feature-split update with the reduce-scattered Adam (pgm_ppo_fs.hip) vs the fp64 oracle's PPO
(a2c_ppo_acktr/algo/ppo.py:58-115: losses, backward, clip_grad_norm_, Adam) at every (parts per tower NS, row tiles
per part R) it runs with: NS = 16 / 8 / 4 / 2 on 4-env minibatches of 256 rows (R = 1 / 2 / 4 / 8), 4 parts on
config 0's 64-row minibatch, the 3-objective critic, and a nonzero entropy coefficient (entered once per tower, also
checked for the row-split kernels the launcher picks by default).  Every task of the launch: parameters, both Adam
moments, the step count and the loss statistics; every update checks the exchange-timeout word."""
import numpy as np
import pytest
import torch

from oracle import ppo as oppo

from .test_gpu_kernels import _close, _update_setup

pytestmark = pytest.mark.gpu


def _check_update(env, P, N, E, M, mb, seed, entropy_coef=0.0, capacity=None, variant=None):
    T = mb * M // N
    args, spec, tb, pols, data, perms = _update_setup(env, P, T, N, E, M, seed=seed, capacity=capacity)
    if variant is not None:
        assert tb.update_variant() == variant
    obs, actions, logp, values, returns, adv = data
    lr = 3e-4
    tb.lr.fill_(lr)
    tb.hp.entropy_coef = entropy_coef
    tb.ppo_update(torch.stack(perms).numpy())
    tb.check_update()
    params, am, av = tb.params.cpu(), tb.adam_m.cpu(), tb.adam_v.cpu()
    steps, stats = tb.adam_step.cpu(), tb.stats.cpu()
    for p in range(P):
        agent = oppo.PPO(pols[p], args.clip_param, E, M, args.value_loss_coef, entropy_coef, lr=lr, eps=1e-5,
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
                st += agent.minibatch_step(*mbt)
        st /= E * M
        ref = tb.layout.flatten(pols[p].state_dict(), dtype=np.float64)
        _close(params[p], ref, 2e-6, 1e-5, f'{env} P={P} task {p}: params')
        m_ref, v_ref, step = tb.layout.adam_from_optimizer_state(agent.optimizer.state_dict()['state'])
        assert int(steps[p]) == step == E * M
        _close(am[p], m_ref, 1e-7, 1e-3, f'{env} task {p}: exp_avg')
        _close(av[p], v_ref, 1e-10, 1e-3, f'{env} task {p}: exp_avg_sq')
        _close(stats[p], st, 1e-5, 1e-4, f'{env} task {p}: loss stats')


# (env, P, N, minibatch rows, two workgroups per CU allowed) -> the launcher's NS: 16 tasks-per-XCD-group rule
# (16 NS ceil(P / 8) <= 256 CUs, or <= 512 with two workgroups per CU where R = 2 fits one CU twice)
@pytest.mark.parametrize('env,P,N,mb,dual', [('MO-Walker2d-v2', 5, 4, 256, '1'),     # NS 16, R 1 (pop 40 over 8 GPUs)
                                             ('MO-Walker2d-v2', 10, 4, 256, '1'),    # NS 8, R 2 (pop 40 / 4: R 1 not doubled)
                                             ('MO-HalfCheetah-v2', 20, 4, 256, '1'),  # NS 8, R 2, 2 per CU (config 2)
                                             ('MO-HalfCheetah-v2', 20, 4, 256, '0'),  # NS 4, R 4
                                             ('MO-Walker2d-v2', 40, 4, 256, '0'),    # NS 2, R 8 (one per CU)
                                             ('MO-Walker2d-v2', 40, 4, 288, '1'),    # NS 6, R 3, 2 per CU
                                             ('MO-Walker2d-v2', 40, 4, 256, '1'),    # NS 6, R 3/3/3/3/2/2, 2 per CU
                                             ('MO-HalfCheetah-v2', 35, 4, 256, '1'),  # the same, a partial group
                                             ('MO-Hopper-v3', 27, 4, 256, '1'),      # NS 8, R 2, 2 per CU, 3 objectives
                                             ('MO-Hopper-v2', 5, 1, 64, '1'),        # NS 4, R 1 (config 0)
                                             ('MO-Ant-v2', 3, 2, 128, '1'),          # NS 8, R 1, O = 27 (two dW1 blocks)
                                             ('MO-Ant-v2', 20, 4, 256, '1'),         # R 2: packed actor loss, A = 8
                                             ('MO-Ant-v2', 40, 4, 256, '1')])        # NS 6, R 3 where it fits
def test_fs_update_all_tasks(gpu, monkeypatch, env, P, N, mb, dual):
    monkeypatch.setenv('PGM_UPDATE_KERNEL', 'fs')
    monkeypatch.setenv('PGM_FS_DUAL', dual)
    _check_update(env, P, N, E=2, M=2, mb=mb, seed=41)  # 4 Adam steps: both slot parities twice


def test_fs_update_capacity_above_active_tasks(gpu, monkeypatch):
    """A batch allocated for 33 task slots running 32 (TaskBatch.set_active): at 32 tasks the feature-split update
    takes 8 parts per tower (16 NS ceil(P / 8) = 512, two per CU), at 33 only 4, and its exchange payload grows with
    NS -- the workspace of the 33-slot batch must hold the 32-task launch's (it was sized by the cap at the
    capacity).  Every task vs the oracle, and the exchange-timeout word."""
    monkeypatch.setenv('PGM_UPDATE_KERNEL', 'fs')
    _check_update('MO-Walker2d-v2', 32, 4, E=1, M=2, mb=256, seed=47, capacity=33,
                  variant='ppo_update_fs_kernel (NS=8, R=2, 2 per CU)')


def test_fs_two_workgroups_per_cu_variant(gpu):
    """The launcher's own description of the dual placement (pgm_ppo_update_variant)."""
    from pgmorl_amd.runtime import TaskBatch
    tb = TaskBatch('MO-HalfCheetah-v2', 20, num_processes=4, num_steps=2048)
    assert tb.update_variant() == 'ppo_update_fs_kernel (NS=8, R=2, 2 per CU)'
    tb = TaskBatch('MO-Walker2d-v2', 5, num_processes=4, num_steps=2048)
    assert tb.update_variant() == 'ppo_update_fs_kernel (NS=16, R=1)'
    tb = TaskBatch('MO-Walker2d-v2', 10, num_processes=4, num_steps=2048)
    assert tb.update_variant() == 'ppo_update_fs_kernel (NS=8, R=2)'
    tb = TaskBatch('MO-Walker2d-v2', 40, num_processes=4, num_steps=2048)  # config 1: 256 rows over 6 parts
    assert tb.update_variant() == 'ppo_update_fs_kernel (NS=6, R=3, 2 per CU)'


@pytest.mark.parametrize('kernel', ['fs', 'default', 'mfma'])
@pytest.mark.parametrize('env,P,N,mb', [('MO-Walker2d-v2', 5, 4, 256), ('MO-Walker2d-v2', 40, 4, 256),
                                        ('MO-Humanoid-v2', 3, 8, 512)])
def test_entropy_coef_enters_once(gpu, monkeypatch, kernel, env, P, N, mb):
    """entropy_coef = 0.01 (ppo.py:98: loss - entropy * entropy_coef): the logstd gradient gets -entropy_coef once
    per tower, whatever the number of row parts and per-workgroup images (t16 NS = 4 at P = 5, MODE 2 at P = 40, the
    wide kernel's NS = 4 for Humanoid, fs NS = 16 / 2)."""
    if kernel == 'fs' and env == 'MO-Humanoid-v2':
        pytest.skip('the feature-split update covers obs_dim <= 32')
    if kernel in ('fs', 'mfma'):  # mfma: the row-split kernels (MODE 2 at P = 40, t16 at P = 5)
        monkeypatch.setenv('PGM_UPDATE_KERNEL', kernel)
    _check_update(env, P, N, E=1, M=2, mb=mb, seed=43, entropy_coef=0.01)
