"""Generate the committed golden vectors under tests/golden/ (run: python -m tests.golden.make_golden).

The reference cannot be run here (standing denial), so these fixtures are produced by
the build's CPU restatement (oracle/, fp64) and by the SynthMO spec generator.  They pin:

  synth_env.npz     every SynthMO env's constants (d, U, c, V, ebase, ecoef, action box, episode length) and
                    reset-state rows for env seeds 0..7 (SURVEY.md §8(d) "committed as fixture arrays")
  kernels.npz       per-seam vectors at Walker dims, seeds 0..2, T=64, N=4, P=3:
                    act (Policy.act, model.py:57-69), gae (storage.py:83-116, 4 flag combos),
                    adv (ppo.py:41-56), ppo (one ppo_epoch x 4 minibatches, ppo.py:58-115), eval (mopg.py:25-46)
  mopg.npz          two full MOPG iterations of one Hopper-v2 task with the reference's RNG draws
                    (torch.manual_seed(j) -> T x normal([N,A]) then E x randperm(T*N); morl/mopg.py:96-135)

Inputs AND outputs are stored, so the GPU tests read only fixtures and the CPU tests re-derive every output from
the oracle to guard it against drift.  Policies are stored as reference state_dict tensors ('<prefix>/<key>').
"""
import argparse
import os

import numpy as np
import torch

from oracle import ppo as oppo
from oracle.mopg import evaluation, initial_sample, mopg_worker
from oracle.policy import make_policy
from oracle.vecenv import RunningMeanStd
from pgmorl_amd import envspec

HERE = os.path.dirname(os.path.abspath(__file__))
F64 = torch.float64
ENV_KEYS = ('d', 'U', 'c', 'V', 'ebase', 'ecoef', 'act_lo', 'act_hi')


def _args(env, **kw):
    spec = envspec.make_spec(env)
    a = dict(env_name=env, obj_num=spec['obj_num'], num_env_steps=10 ** 9, seed=0, num_steps=64,
             num_processes=4, ppo_epoch=1, num_mini_batch=4, clip_param=0.2, value_loss_coef=0.5,
             entropy_coef=0.0, lr=3e-4, max_grad_norm=0.5, gamma=0.995, gae_lambda=0.95, use_gae=True,
             use_proper_time_limits=True, ob_rms=True, obj_rms=True, raw=True, eval_num=1,
             use_linear_lr_decay=True, lr_decay_ratio=1.0, layernorm=False)
    a.update(kw)
    return argparse.Namespace(**a)


def _policy(spec, seed, scale):
    """Reference-initialised policy, perturbed (breaks zero bias / zero logstd), rounded to fp32 values."""
    torch.manual_seed(seed)
    pol = make_policy(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
    g = torch.Generator().manual_seed(seed + 100)
    with torch.no_grad():
        for prm in pol.parameters():
            prm.add_(torch.randn(prm.shape, generator=g, dtype=F64) * scale)
            prm.copy_(prm.float().double())
    return pol


def _put_policy(out, prefix, pol):
    for k, v in pol.state_dict().items():
        out[f'{prefix}/{k}'] = v.numpy().copy()


def synth_env():
    out = {}
    for name in envspec.env_names():
        s = envspec.make_spec(name)
        for k in ENV_KEYS:
            out[f'{name}/{k}'] = s[k]
        out[f'{name}/dims'] = np.array([s['obs_dim'], s['act_dim'], s['obj_num'], s['max_episode_steps']])
        out[f'{name}/s0'] = envspec.reset_table(s['obs_dim'], 0, 8)
    return out


def kernels():
    env, P, T, N = 'MO-Walker2d-v2', 3, 64, 4
    spec = envspec.make_spec(env)
    O, A, K = spec['obs_dim'], spec['act_dim'], spec['obj_num']
    out = {'dims': np.array([P, T, N, O, A, K])}
    rng = np.random.RandomState(20261015)
    pols = [_policy(spec, p, 0.05) for p in range(P)]
    for p, pol in enumerate(pols):
        _put_policy(out, f'pol{p}', pol)
    # act: obs [P][N][O] fp32 values, shared noise [N][A]
    obs = rng.randn(P, N, O).astype(np.float32)
    noise = rng.randn(N, A).astype(np.float32)
    out['act/obs'], out['act/noise'] = obs, noise
    for p, pol in enumerate(pols):
        with torch.no_grad():
            v, a, lp = pol.act(torch.from_numpy(obs[p]).double(), noise=torch.from_numpy(noise).double())
            _, am, _ = pol.act(torch.from_numpy(obs[p]).double(), deterministic=True)
        out[f'act/value{p}'], out[f'act/action{p}'] = v.numpy(), a.numpy()
        out[f'act/logp{p}'], out[f'act/mean{p}'] = lp[:, 0].numpy(), am.numpy()
    # gae: random storage with episode ends and time-limit ends
    rew = rng.randn(P, T, N, K).astype(np.float32)
    val = rng.randn(P, T + 1, N, K).astype(np.float32)
    masks = np.ones((P, T + 1, N), np.float32)
    bad = np.ones((P, T + 1, N), np.float32)
    done = rng.rand(P, T + 1, N) < 0.06
    masks[done] = 0.0
    bad[done & (rng.rand(P, T + 1, N) < 0.5)] = 0.0
    out['gae/rewards'], out['gae/values'], out['gae/masks'], out['gae/bad_masks'] = rew, val, masks, bad
    for use_gae in (0, 1):
        for proper in (0, 1):
            r = np.zeros((P, T + 1, N, K))
            for p in range(P):
                ret = torch.zeros(T + 1, N, K, dtype=F64)
                v = torch.from_numpy(val[p]).double()
                oppo.compute_returns_inplace(torch.from_numpy(rew[p]).double(), v.clone(),
                                             torch.from_numpy(masks[p]).double().unsqueeze(-1),
                                             torch.from_numpy(bad[p]).double().unsqueeze(-1), ret, v[-1],
                                             bool(use_gae), 0.99, 0.95, bool(proper))
                r[p] = ret.numpy()
            out[f'gae/returns_g{use_gae}_p{proper}'] = r
    # adv: returns/values -> normalised scalarised advantages
    R = (rng.randn(P, T + 1, N, K) * 3 + 1).astype(np.float32)
    V = (rng.randn(P, T + 1, N, K) * 2).astype(np.float32)
    w = rng.dirichlet(np.ones(K), size=P)
    var = rng.rand(P, K) * 4 + 0.1
    out['adv/returns'], out['adv/values'], out['adv/weights'], out['adv/obj_var'] = R, V, w, var
    out['adv/adv'] = np.stack([oppo.scalarized_normalized_advantages(
        torch.from_numpy(R[p]).double(), torch.from_numpy(V[p]).double(), w[p], var[p]).numpy() for p in range(P)])
    out['adv/adv_noobjrms'] = np.stack([oppo.scalarized_normalized_advantages(
        torch.from_numpy(R[p]).double(), torch.from_numpy(V[p]).double(), w[p], None).numpy() for p in range(P)])
    # ppo: one epoch x 4 minibatches on a consistent rollout (actions/logp/values from the policy, perturbed)
    E, M, lr = 1, 4, 3e-4
    B = T * N
    xo = np.clip(rng.randn(P, T + 1, N, O), -3, 3).astype(np.float32)
    perms = np.stack([np.random.RandomState(77 + e).permutation(B) for e in range(E)]).astype(np.int32)
    out['ppo/obs'], out['ppo/perms'], out['ppo/lr'] = xo, perms, np.array(lr)
    acts, lps, vals, rets, advs = [], [], [], [], []
    for p, pol in enumerate(pols):
        eps = rng.randn(T, N, A)
        with torch.no_grad():
            v, a, lp = pol.act(torch.from_numpy(xo[p, :T]).double().reshape(B, O),
                               noise=torch.from_numpy(eps).reshape(B, A))
        acts.append(a.float().reshape(T, N, A).numpy())
        lps.append((lp[:, 0].numpy() + rng.randn(B) * 0.05).astype(np.float32).reshape(T, N))
        vv = (v.numpy() + rng.randn(B, K) * 0.1).astype(np.float32).reshape(T, N, K)
        vals.append(np.concatenate([vv, np.zeros((1, N, K), np.float32)]))
        rets.append((vals[-1] + rng.randn(T + 1, N, K) * 0.5).astype(np.float32))
        advs.append(rng.randn(T, N).astype(np.float32))
    out['ppo/actions'], out['ppo/logp'] = np.stack(acts), np.stack(lps)
    out['ppo/values'], out['ppo/returns'], out['ppo/adv'] = np.stack(vals), np.stack(rets), np.stack(advs)
    args = _args(env, num_steps=T, num_processes=N, ppo_epoch=E, num_mini_batch=M)
    for p in range(P):
        pol = _policy(spec, p, 0.05)
        agent = oppo.PPO(pol, args.clip_param, E, M, args.value_loss_coef, args.entropy_coef, lr=lr, eps=1e-5,
                         max_grad_norm=args.max_grad_norm)
        ro = oppo.RolloutStorage(T, N, O, A, K)
        ro.obs.copy_(torch.from_numpy(xo[p]).double())
        ro.actions.copy_(torch.from_numpy(acts[p]).double())
        ro.action_log_probs.copy_(torch.from_numpy(lps[p]).double().unsqueeze(-1))
        ro.value_preds.copy_(torch.from_numpy(vals[p]).double())
        ro.returns.copy_(torch.from_numpy(rets[p]).double())
        stats = np.zeros(3)
        for e in range(E):
            for mbt in ro.minibatches(torch.from_numpy(advs[p]).double(), M, torch.from_numpy(perms[e]).long()):
                stats += agent.minibatch_step(*mbt)
        _put_policy(out, f'ppo/after{p}', pol)
        st = agent.optimizer.state_dict()['state']
        names = [k for k, _ in pol.named_parameters()]
        for i, k in enumerate(names):
            out[f'ppo/exp_avg{p}/{k}'] = st[i]['exp_avg'].numpy().copy()
            out[f'ppo/exp_avg_sq{p}/{k}'] = st[i]['exp_avg_sq'].numpy().copy()
        out[f'ppo/stats{p}'] = stats / (E * M)
    # eval: deterministic episode from fixed ob_rms
    s0_eval = envspec.reset_table(O, 0, 1)
    args = _args(env, eval_num=1, raw=True)
    for p, pol in enumerate(pols):
        r = RunningMeanStd(shape=(O,))
        r.update(rng.randn(50, O) * 0.3 + 0.1)
        out[f'eval/ob_mean{p}'], out[f'eval/ob_var{p}'], out[f'eval/ob_count{p}'] = r.mean, r.var, np.array(r.count)
        out[f'eval/objs{p}'] = evaluation(args, spec, s0_eval, pol, r)
    return out


def host_draws(T, N, A, E):
    """The reference's per-iteration RNG draws (morl/mopg.py:96 reseed; distributions.py:30-40 normal;
    storage.py:133-136 randperm)."""
    def fn(j):
        torch.manual_seed(j)
        noise = torch.stack([torch.normal(torch.zeros(N, A, dtype=F64), torch.ones(N, A, dtype=F64))
                             for _ in range(T)])
        return noise, [torch.randperm(T * N) for _ in range(E)]
    return fn


def mopg():
    env, T, N, E, M, iters = 'MO-Hopper-v2', 64, 4, 2, 4, 2
    spec = envspec.make_spec(env)
    args = _args(env, num_steps=T, num_processes=N, ppo_epoch=E, num_mini_batch=M, num_env_steps=T * N * 10)
    torch.manual_seed(0)
    sample = initial_sample(args, spec)
    with torch.no_grad():
        for prm in sample.actor_critic.parameters():
            prm.copy_(prm.float().double())
    w = np.array([0.3, 0.7])
    out = {'dims': np.array([T, N, E, M, iters]), 'weights': w, 'num_env_steps': np.array(args.num_env_steps)}
    _put_policy(out, 'init', sample.actor_critic)
    fn = host_draws(T, N, spec['act_dim'], E)
    for j in range(iters):
        noise, perms = fn(j)
        out[f'it{j}/noise'] = noise.float().numpy()
        out[f'it{j}/perms'] = torch.stack(perms).numpy().astype(np.int32)

    def fn32(j):  # the device consumes the fp32-rounded normal draws
        noise, perms = fn(j)
        return noise.float().double(), perms

    record = []
    s0_train = envspec.reset_table(spec['obs_dim'], 0, N)
    s0_eval = envspec.reset_table(spec['obs_dim'], 0, 1)
    offs = mopg_worker(args, spec, s0_train, s0_eval, sample, w, 0, iters, noise_fn=fn32, record=record)
    for j, (off, rec) in enumerate(zip(offs, record)):
        _put_policy(out, f'it{j}/params', off.actor_critic)
        out[f'it{j}/objs'] = off.objs
        out[f'it{j}/stats'] = np.asarray(rec['stats'])
        out[f'it{j}/obj_var'] = rec['obj_var']
        for k in ('obs', 'actions', 'value_preds', 'rewards', 'returns'):
            out[f'it{j}/{k}'] = rec[k].numpy()
        for k in ('action_log_probs', 'masks', 'bad_masks'):
            out[f'it{j}/{k}'] = rec[k][..., 0].numpy()
        ep = off.env_params
        out[f'it{j}/ob_mean'], out[f'it{j}/ob_var'] = ep['ob_rms'].mean, ep['ob_rms'].var
        out[f'it{j}/obj_mean'], out[f'it{j}/obj_var_end'] = ep['obj_rms'].mean, ep['obj_rms'].var
    return out


def main():
    torch.set_num_threads(1)
    for name, fn in (('synth_env', synth_env), ('kernels', kernels), ('mopg', mopg)):
        path = os.path.join(HERE, name + '.npz')
        np.savez_compressed(path, **fn())
        print(path, os.path.getsize(path), 'bytes')


if __name__ == '__main__':
    main()
