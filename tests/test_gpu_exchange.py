"""The update kernels' cross-workgroup exchanges under provoked delays, and the launcher's co-residency check.

Every row-split update (MODE 2: each tower on two workgroups; t16: on four) hands gradient images over through
16-B sc1 publishes + tagged flag granules, and the two towers hand their squared norms over through tagged 8-B
granules, all double-buffered by Adam-step parity (pgm_common.hpp ppo_norm_granule).  PGM_TEST_DELAY (read only by
the test build libpgm_test.so, -DPGM_TEST_HOOKS, which these tests run through _lib.test_build()) stalls ONE
workgroup for a fixed number of cycles at one hand-off point of one step:
  where 0 -- before it publishes its gradient image (its partners spin on its flag),
  where 1 -- between its image flag store and its own partner poll (the partners run ahead to the next step),
  where 2 -- between its tower-norm granule store and its poll: the other tower can finish this step and
             publish the NEXT step's norm before the delayed poll looks -- the order a single-buffered granule
             lost (the poll would see the next tag and spin until the timeout word).
  where 3 -- (feature-split update only) before its Adam step and parameter publish.
Each case must leave the exchange-timeout word clear (check_update) and the parameters equal to the oracle's.
"""
import numpy as np
import pytest
import torch

from oracle import ppo as oppo
from pgmorl_amd import _lib
from pgmorl_amd._lib import PGMError

from .test_gpu_kernels import _close, _update_setup

pytestmark = pytest.mark.gpu

DELAY = 4_000_000  # shader cycles (~2 ms): far beyond one Adam step, far below the 2^26-spin timeout


def _run_update(env, P, T, N, E, M, split, delay, monkeypatch):
    if split == 'fs':
        monkeypatch.setenv('PGM_UPDATE_KERNEL', 'fs')
    else:
        monkeypatch.setenv('PGM_UPDATE_SPLIT', split)
    if delay is not None:
        monkeypatch.setenv('PGM_TEST_DELAY', ':'.join(str(x) for x in delay))
    args, spec, tb, pols, data, perms = _update_setup(env, P, T, N, E, M, seed=17)
    obs, actions, logp, values, returns, adv = data
    lr = 3e-4
    tb.lr.fill_(lr)
    with _lib.test_build():
        tb.ppo_update(torch.stack(perms).numpy())
    tb.check_update()  # PGMError if any spin-wait gave up
    for p in range(P):
        agent = oppo.PPO(pols[p], args.clip_param, E, M, args.value_loss_coef, args.entropy_coef, lr=lr, eps=1e-5,
                         max_grad_norm=args.max_grad_norm)
        ro = oppo.RolloutStorage(T, N, spec['obs_dim'], spec['act_dim'], spec['obj_num'])
        ro.obs.copy_(torch.from_numpy(obs[p]).double())
        ro.actions.copy_(actions[p].double())
        ro.action_log_probs.copy_(logp[p].double().unsqueeze(-1))
        ro.value_preds.copy_(values[p].double())
        ro.returns.copy_(returns[p].double())
        for e in range(E):
            for mbt in ro.minibatches(adv[p].double(), M, perms[e]):
                agent.minibatch_step(*mbt)
        _close(tb.params[p].cpu(), tb.layout.flatten(pols[p].state_dict(), dtype=np.float64), 2e-6, 1e-5,
               f'task {p}: params with delay {delay}')
        assert int(tb.adam_step[p]) == E * M


def block_of(kernel, task, tower, part, ns=4):
    """blockIdx.x of (task, tower 0 = critic / 1 = actor, row part) under the HEAD block maps: every workgroup of a
    task on blocks b, b + 8, ... (one XCD) -- MODE 2 (pgm_ppo_mfma.hip ppo_update_mfma_kernel): groups
    of 32 blocks per 8 tasks, block r = half (r >> 4) & 1 of tower (r >> 3) & 1 of task 8 G + (r & 7); t16 (NS = 4)
    and the feature-split kernel (pgm_ppo_fs.hip, NS parts): groups of 16 NS blocks per 8 tasks, block r = part
    ((r >> 3) % 2 NS) >> 1 of tower (r >> 3) & 1 of task 8 G + (r & 7)."""
    if kernel == '2':
        return 32 * (task // 8) + 16 * part + 8 * tower + (task & 7)
    return 16 * ns * (task // 8) + 8 * (2 * part + tower) + (task & 7)


def test_block_of_inverts_the_kernel_maps():
    for kernel, ns in (('2', 2), ('4', 4), ('fs', 16), ('fs', 2)):
        seen = set()
        for task in range(11):
            for tower in (0, 1):
                for part in range(ns):
                    b = block_of(kernel, task, tower, part, ns)
                    if kernel == '2':
                        got = (8 * (b >> 5) + (b & 7), (b >> 3) & 1, (b >> 4) & 1)
                    else:
                        j = (b >> 3) % (2 * ns)
                        got = (8 * (b // (16 * ns)) + (b & 7), j & 1, j >> 1)
                    assert got == (task, tower, part) and b not in seen
                    seen.add(b)


# (kernel, task, tower, part, where): stall that workgroup at that hand-off; fs: NS = 16 parts for 2 Walker tasks,
# where 3 = before its Adam / parameter publish
CASES = [('2', 0, 0, 0, 0), ('2', 0, 1, 1, 0), ('2', 0, 0, 1, 1), ('2', 0, 1, 0, 1), ('2', 0, 0, 0, 2), ('2', 0, 1, 1, 2),
         ('4', 0, 0, 0, 0), ('4', 0, 1, 3, 0), ('4', 0, 1, 2, 1), ('4', 0, 0, 0, 2), ('4', 0, 1, 0, 2), ('4', 0, 0, 3, 2),
         ('fs', 0, 0, 0, 0), ('fs', 1, 1, 15, 0), ('fs', 0, 1, 7, 1), ('fs', 1, 0, 3, 2), ('fs', 0, 1, 0, 2),
         ('fs', 1, 1, 9, 3), ('fs', 0, 0, 15, 3)]


@pytest.mark.parametrize('split,task,tower,part,where', CASES)
def test_delayed_handoff_keeps_parity(gpu, split, task, tower, part, where, monkeypatch):
    # Walker, 2 tasks, mb = 256 (the single-tile specialisations of MODE 2 / t16; fs: 16 parts of one 16-row tile),
    # 4 Adam steps; the stall hits step 1 (both parities are exercised before and after it)
    block = block_of(split, task, tower, part, 16 if split == 'fs' else 4)
    _run_update('MO-Walker2d-v2', 2, 256, 4, 1, 4, split, (1, block, where, DELAY), monkeypatch)


@pytest.mark.parametrize('split', ['2', '4', 'fs'])
def test_delay_on_last_step_and_ragged_grid(gpu, split, monkeypatch):
    # Hopper-v3 (3 objectives), 5 tasks (a partial group of 8 tasks in the block map), multi-pass minibatches for
    # MODE 2 / t16 (mb = 128 with N = 2: not the single-tile path; fs: 8 parts of one tile); stall the last task's
    # actor part 0 on the last step
    P = 5
    block = block_of(split, P - 1, 1, 0, 8 if split == 'fs' else 4)
    _run_update('MO-Hopper-v3', P, 128, 2, 1, 2, split, (1, block, 2, DELAY), monkeypatch)


@pytest.mark.parametrize('task,tower,part,where', [(19, 1, 7, 1), (0, 0, 0, 3), (13, 1, 4, 2), (8, 0, 3, 0)])
def test_delay_two_workgroups_per_cu(gpu, task, tower, part, where, monkeypatch):
    # Walker P = 20 with 8 parts per tower of two 16-row tiles: 384 workgroups, two per CU where they share one
    # (fs_choose_ns dual); a stalled workgroup may share its CU with another task's part while its partners spin
    monkeypatch.setenv('PGM_FS_DUAL', '1')
    block = block_of('fs', task, tower, part, 8)
    _run_update('MO-Walker2d-v2', 20, 256, 4, 1, 4, 'fs', (1, block, where, DELAY), monkeypatch)


@pytest.mark.parametrize('task,tower,part,where', [(39, 1, 5, 1), (0, 0, 0, 3), (21, 1, 3, 2), (34, 0, 4, 0)])
def test_delay_six_ragged_parts(gpu, task, tower, part, where, monkeypatch):
    # Walker P = 40, 256-row minibatches over 6 parts of 3 / 3 / 3 / 3 / 2 / 2 row tiles (dummy tiles in parts 4, 5):
    # 480 workgroups, two per CU; stalls in a 3-tile and in a 2-tile part
    block = block_of('fs', task, tower, part, 6)
    _run_update('MO-Walker2d-v2', 40, 256, 4, 1, 4, 'fs', (1, block, where, DELAY), monkeypatch)


def test_coresidency_check_refuses_an_oversized_grid(gpu, monkeypatch):
    """The launcher refuses (PGM_E_UNSUPPORTED -> PGMError) a grid whose workgroups cannot all be resident:
    PGM_TEST_RESIDENT_CUS pretends the device has fewer CUs than the grid's workgroups (one per CU)."""
    monkeypatch.setenv('PGM_UPDATE_SPLIT', '2')
    # MODE 2 grid for 2 tasks: one group of 8 tasks' blocks (32 workgroups, 8 of them live; padding exits at once)
    monkeypatch.setenv('PGM_TEST_RESIDENT_CUS', '16')
    args, spec, tb, pols, data, perms = _update_setup('MO-Walker2d-v2', 2, 64, 4, 1, 1, seed=3)
    with _lib.test_build():
        with pytest.raises(PGMError, match='co-resident'):
            tb.ppo_update(torch.stack(perms).numpy())
        monkeypatch.setenv('PGM_TEST_RESIDENT_CUS', '32')  # exactly fits: runs
        tb.ppo_update(torch.stack(perms).numpy())
    tb.check_update()
    # the production library has no such hook: the same override changes nothing there
    monkeypatch.setenv('PGM_TEST_RESIDENT_CUS', '16')
    tb.ppo_update(torch.stack(perms).numpy())
    tb.check_update()
