"""Parity at the PRODUCTION per-GPU populations of every BASELINE.json config (MI355X, fp32, vs the fp64 CPU
oracle), with short horizons so the oracle finishes in seconds:

  * MO-Walker2d-v2   P = 40            (config 1: one GPU; the feature-split update on 6 parts per tower,
                                         ragged 3 / 3 / 3 / 3 / 2 / 2 row tiles, 480 workgroups two per CU)
  * MO-HalfCheetah-v2 P = 20           (config 2: pop 160 sharded over 8 GPUs; feature-split, 8 parts, two per CU)
  * MO-Hopper-v3     P = 27, 3 objectives (config 3: pop 210 over 8 GPUs -> blocks of 27 / 26; a partial last
                                         group of 8 tasks in the block map; feature-split, 8 parts, two per CU)
  * MO-Humanoid-v2   P = 20, N = 8     (config 4: pop 160 over 8 GPUs; wide update = 80 workgroups,
                                         minibatch 512 rows as in production)

Every task of the launch is compared (not a subset), and every update checks the exchange-timeout word
through TaskBatch.check_update (PGMError if a spin-wait gave up).  Minibatch shapes are the production
ones (mb = T*N/32 = 256 rows for N = 4, 512 for Humanoid's N = 8): T and M are cut together.
"""
import numpy as np
import pytest
import torch

from oracle import ppo as oppo
from oracle.mopg import initial_sample, mopg_worker
from oracle.vecenv import VecNormalizedSynth
from pgmorl_amd import envspec
from pgmorl_amd.runtime import TaskBatch

from .helpers import small_args, weights_grid
from .test_gpu_kernels import (_batch_with_policies, _close, _noise_fn, _oracle_rollout, _teacher_forced_check,
                               _update_setup)

pytestmark = pytest.mark.gpu

CONFIGS = [('MO-Hopper-v2', 5, 1), ('MO-Walker2d-v2', 40, 4), ('MO-HalfCheetah-v2', 20, 4), ('MO-Hopper-v3', 27, 4),
           ('MO-Humanoid-v2', 20, 8)]
MB = {1: 64, 4: 256, 8: 512}  # production minibatch rows T * N / 32 (config 0 runs N = 1: 64 rows)


@pytest.mark.parametrize('env,P,N', CONFIGS)
def test_production_update_all_tasks(gpu, env, P, N):
    """One launch of pgm_ppo_update over the whole per-GPU population, 2 Adam steps of a production-size
    minibatch (mb = 256 / 512 rows); parameters, Adam moments, step and loss stats of EVERY task."""
    mb = MB[N]
    M, E = 2, 1
    T = mb * M // N
    args, spec, tb, pols, data, perms = _update_setup(env, P, T, N, E, M, seed=21)
    obs, actions, logp, values, returns, adv = data
    lr = 3e-4
    tb.lr.fill_(lr)
    tb.ppo_update(torch.stack(perms).numpy())
    tb.check_update()
    params, am, av = tb.params.cpu(), tb.adam_m.cpu(), tb.adam_v.cpu()
    steps, stats = tb.adam_step.cpu(), tb.stats.cpu()
    for p in range(P):
        agent = oppo.PPO(pols[p], args.clip_param, E, M, args.value_loss_coef, args.entropy_coef, lr=lr, eps=1e-5,
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
        _close(params[p], ref, 2e-6, 1e-5, f'{env} task {p}/{P}: params')
        m_ref, v_ref, step = tb.layout.adam_from_optimizer_state(agent.optimizer.state_dict()['state'])
        assert int(steps[p]) == step == E * M
        _close(am[p], m_ref, 1e-7, 1e-3, f'{env} task {p}: exp_avg')
        _close(av[p], v_ref, 1e-10, 1e-3, f'{env} task {p}: exp_avg_sq')
        _close(stats[p], st, 1e-5, 1e-4, f'{env} task {p}: loss stats')


@pytest.mark.parametrize('env,P,N', CONFIGS)
def test_production_rollout_all_tasks(gpu, env, P, N):
    """The rollout kernel over the whole per-GPU population (one workgroup per task), every task vs the oracle
    VecNormalized env + policy (Humanoid teacher-forced, see test_gpu_kernels.test_rollout)."""
    T = 40
    spec, tb, pols = _batch_with_policies(env, P, N, T, seed=9, scale=0.05)
    s0 = envspec.reset_table(spec['obs_dim'], 0, N)
    noise = torch.randn(T, N, spec['act_dim'], generator=torch.Generator().manual_seed(10), dtype=torch.float64)
    tb.env_reset()
    tb.rollout(0, noise=noise.float(), carry=False)
    if spec['obs_dim'] > 48:
        for p in range(P):
            _teacher_forced_check(tb, p, pols[p], spec, s0, noise)
        return
    obs, acts, lps, vals = tb.obs.cpu(), tb.actions.cpu(), tb.logp.cpu(), tb.values.cpu()
    rews, masks = tb.rewards.cpu(), tb.masks.cpu().numpy()
    for p in range(P):
        envs = VecNormalizedSynth(spec, s0, 0.995)
        ro = oppo.RolloutStorage(T, N, spec['obs_dim'], spec['act_dim'], spec['obj_num'])
        ro.obs[0].copy_(torch.from_numpy(envs.reset()).double())
        _oracle_rollout(pols[p], envs, ro, noise.float().double())
        _close(obs[p], ro.obs, 5e-5, 1e-4, f'{env} task {p}: obs')
        _close(acts[p], ro.actions, 5e-5, 1e-4, f'{env} task {p}: actions')
        _close(lps[p], ro.action_log_probs[..., 0], 2e-4, 1e-4, f'{env} task {p}: logp')
        _close(vals[p], ro.value_preds, 5e-5, 1e-4, f'{env} task {p}: values')
        _close(rews[p], ro.rewards, 5e-5, 1e-4, f'{env} task {p}: rewards')
        np.testing.assert_array_equal(masks[p], ro.masks[..., 0].numpy())


@pytest.mark.parametrize('env,P,N', [('MO-Walker2d-v2', 40, 4), ('MO-Hopper-v3', 27, 4), ('MO-Hopper-v2', 5, 1)])
def test_production_iteration(gpu, env, P, N):
    """A full MOPG iteration (rollout, GAE, advantages, the update kernel the launcher picks for this P -- the
    feature-split update on 6 parts per tower for Walker P = 40 (mb = 256: ragged 3 / 3 / 3 / 3 / 2 / 2 row tiles), on 8
    parts two per CU for Hopper-v3 P = 27, on 4 parts for config 0's Hopper-v2 P = 5 (mb = 64) -- and the
    evaluation) at the production population with the reference's RNG draws; tasks spread over the grid vs the
    oracle MOPG_worker (morl/mopg.py:60-182)."""
    T, E, M = 64, 1, 1  # one production-size minibatch (mb = T * N: 256 rows, config 0's N = 1: 64), one Adam step
    args = small_args(env, num_steps=T, num_processes=N, ppo_epoch=E, num_mini_batch=M, num_env_steps=T * N * 10)
    spec = envspec.make_spec(env)
    A, B = spec['act_dim'], T * N
    tb = TaskBatch(env, P, num_processes=N, num_steps=T, ppo_epoch=E, num_mini_batch=M)
    fn = _noise_fn(T, N, A, E, B)
    w = weights_grid(spec['obj_num'], P)
    torch.manual_seed(0)
    samples = [initial_sample(args, spec) for _ in range(P)]
    for s in samples:
        with torch.no_grad():
            for prm in s.actor_critic.parameters():
                prm.copy_(prm.float().double())
    for p, s in enumerate(samples):
        tb.set_task(p, s.actor_critic.state_dict(), {}, s.env_params, w[p])
    tb.env_reset()
    total = int(args.num_env_steps) // T // N
    noise, perms = fn(0)
    tb.iteration(0, oppo.linear_lr(0, total, args.lr), noise=noise.float(), perms=torch.stack(perms).numpy(),
                 carry=False)
    tb.check_update()
    objs, params = tb.objs.cpu().numpy(), tb.params.cpu().numpy()
    s0_train = envspec.reset_table(spec['obs_dim'], 0, N)
    s0_eval = envspec.reset_table(spec['obs_dim'], 0, 1)
    for p in sorted({0, 1, P // 3, P // 2, P - 2, P - 1}):
        off = mopg_worker(args, spec, s0_train, s0_eval, samples[p], w[p], 0, 1, noise_fn=fn)[0]
        _close(params[p], tb.layout.flatten(off.actor_critic.state_dict(), dtype=np.float64), 2e-5, 1e-4,
               f'{env} task {p}/{P}: params')
        _close(objs[p], off.objs, 1e-3, 1e-4, f'{env} task {p}: eval objs')


@pytest.mark.parametrize('env,P,eval_num', [('MO-Hopper-v2', 5, 1), ('MO-Walker2d-v2', 40, 1), ('MO-HalfCheetah-v2', 20, 1),
                                             ('MO-Hopper-v3', 27, 2), ('MO-Humanoid-v2', 20, 6)])
def test_production_eval_all_tasks(gpu, env, P, eval_num):
    """pgm_eval over the production population (Humanoid: eval_num 6, scripts/humanoid-v2.py:45), every task.

    Deterministic 500-step episodes can be chaotic: for some policies of this population a 1e-7 relative
    change of the parameters moves the objective sums of SynthMO-Walker by ~11 (measured with the fp64
    oracle alone), so whole-episode fp32-vs-fp64 sums are not comparable for every task (full-length
    episodes are checked on non-chaotic tasks by test_gpu_kernels.test_eval and after a real update by
    test_production_iteration).  Here every episode is cut to 12 steps on both sides (the time limit is a
    field of the env spec), where the oracle's own fp32 twin (torch fp32 policy) stays within 1.8e-6
    relative (1.5e-5 for Humanoid's 376-input policy) on all tasks; the device must match to
    1e-4 + 2e-5 |ref| (Humanoid 1e-3 + 2e-4 |ref|)."""
    from oracle.mopg import evaluation as oracle_evaluation
    from oracle.vecenv import RunningMeanStd
    spec, tb, pols = _batch_with_policies(env, P, 4, 8, seed=5, scale=0.1, eval_num=eval_num)
    spec = dict(spec, max_episode_steps=12)
    tb.spec = spec
    tb.c_spec.max_episode_steps = 12
    args = small_args(env, eval_num=eval_num)
    rng = np.random.RandomState(2)
    rms = []
    for p in range(P):
        r = RunningMeanStd(shape=(spec['obs_dim'],))
        r.update(rng.randn(50, spec['obs_dim']) * 0.3 + 0.1)
        rms.append(r)
        tb.set_env_params(p, {'ob_rms': r})
    objs = tb.evaluate().cpu().numpy()
    s0_eval = envspec.reset_table(spec['obs_dim'], 0, eval_num)
    atol, rtol = (1e-4, 2e-5) if spec['obs_dim'] <= 48 else (1e-3, 2e-4)
    for p in range(P):
        _close(objs[p], oracle_evaluation(args, spec, s0_eval, pols[p], rms[p]), atol, rtol, f'{env} task {p}: objs')


def test_config0_full_iteration_shape(gpu):
    """Config 0 at its real shape -- Hopper-v2, P = 5, N = 1, T = 2048, M = 32 (minibatch 64: the feature-split update
    on 4 parts per tower, one 16-row tile each), two epochs -- one launch of pgm_ppo_update
    for every task vs the oracle, then a full TaskBatch.iteration (rollout of 2,048 steps, GAE, advantages, that
    update, evaluation) for every task vs oracle.mopg.mopg_worker (scripts/hopper-v2.py:38, morl/mopg.py:60-182)."""
    env, P, N, T, E, M = 'MO-Hopper-v2', 5, 1, 2048, 2, 32
    args, spec, tb, pols, data, perms = _update_setup(env, P, T, N, E, M, seed=31)
    obs, actions, logp, values, returns, adv = data
    lr = 3e-4
    tb.lr.fill_(lr)
    tb.ppo_update(torch.stack(perms).numpy())
    tb.check_update()
    params, steps = tb.params.cpu(), tb.adam_step.cpu()
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
        assert int(steps[p]) == E * M
        _close(params[p], tb.layout.flatten(pols[p].state_dict(), dtype=np.float64), 5e-6, 1e-4,
               f'config 0 task {p}: params after {E * M} Adam steps')
    # the whole iteration at the production shape (one epoch: the oracle's 2,048-step rollout dominates)
    E = 1
    args = small_args(env, num_steps=T, num_processes=N, ppo_epoch=E, num_mini_batch=M, num_env_steps=T * N * 10)
    A, B = spec['act_dim'], T * N
    tb = TaskBatch(env, P, num_processes=N, num_steps=T, ppo_epoch=E, num_mini_batch=M)
    fn = _noise_fn(T, N, A, E, B)
    w = weights_grid(spec['obj_num'], P)
    torch.manual_seed(0)
    samples = [initial_sample(args, spec) for _ in range(P)]
    for s in samples:
        with torch.no_grad():
            for prm in s.actor_critic.parameters():
                prm.copy_(prm.float().double())
    for p, s in enumerate(samples):
        tb.set_task(p, s.actor_critic.state_dict(), {}, s.env_params, w[p])
    tb.env_reset()
    total = int(args.num_env_steps) // T // N
    noise, perms = fn(0)
    tb.iteration(0, oppo.linear_lr(0, total, args.lr), noise=noise.float(), perms=torch.stack(perms).numpy(),
                 carry=False)
    tb.check_update()
    objs, params = tb.objs.cpu().numpy(), tb.params.cpu().numpy()
    s0_train = envspec.reset_table(spec['obs_dim'], 0, N)
    s0_eval = envspec.reset_table(spec['obs_dim'], 0, 1)
    for p in range(P):
        off = mopg_worker(args, spec, s0_train, s0_eval, samples[p], w[p], 0, 1, noise_fn=fn)[0]
        _close(params[p], tb.layout.flatten(off.actor_critic.state_dict(), dtype=np.float64), 5e-5, 1e-3,
               f'config 0 task {p}: params after a full iteration')
        _close(objs[p], off.objs, 1e-2, 1e-4, f'config 0 task {p}: eval objs')
