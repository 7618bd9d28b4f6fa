"""Oracle: the MOPG task loop and deterministic evaluation (CPU, fp64).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates:
  * MOPG_worker (per-task PPO iterations, RNG reseed per iteration, linear LR,
    rollout T x N, bootstrap value, GAE, scalarised update, after_update,
    snapshot + evaluation every iteration)            -- morl/mopg.py:60-182
  * evaluation (fresh env seeded seed+eval_id, obs normalised by the snapshot
    ob_rms WITHOUT the float32 round, deterministic action, raw objective sum)
                                                       -- morl/mopg.py:25-46
  * Sample (env_params + policy + optimizer state)     -- morl/sample.py:10-32

The MuJoCo envs are replaced by the synthetic env of oracle/vecenv.py; multiprocessing
fan-out is replaced by a plain loop over tasks (tasks never interact inside a generation).
"""
import copy
import os
import time

import numpy as np
import torch

from .policy import make_policy
from .ppo import PPO, RolloutStorage, linear_lr
from .vecenv import RunningMeanStd, SynthEnv, VecNormalizedSynth

F64 = torch.float64
# Precision arm of scripts/hv_full.py (PGM_ORACLE_NET_DTYPE=float32): the policy, its PPO losses / backward / Adam in
# fp32 (the device's arithmetic), the envs, running statistics and returns still fp64.  Default: the fp64 reference.
NET = torch.float32 if os.environ.get('PGM_ORACLE_NET_DTYPE') == 'float32' else F64


def _to_net_dtype(policy, agent):
    """Cast a sample's policy and Adam state to NET in place (no-op for fp64)."""
    if NET == F64:
        return
    policy.to(NET)
    for st in agent.optimizer.state.values():
        for k in ('exp_avg', 'exp_avg_sq'):
            if k in st:
                st[k] = st[k].to(NET)


class OracleSample:
    """Sample = (env_params, actor_critic, agent, objs, optgraph_id) (morl/sample.py)."""

    def __init__(self, env_params, actor_critic, agent, objs=None, optgraph_id=None):
        self.env_params, self.actor_critic, self.agent = env_params, actor_critic, agent
        self.agent.actor_critic = actor_critic
        state = copy.deepcopy(agent.optimizer.state_dict())
        agent.optimizer = torch.optim.Adam(actor_critic.parameters(), lr=3e-4, eps=1e-5)
        agent.optimizer.load_state_dict(state)
        self.objs, self.optgraph_id = objs, optgraph_id

    @classmethod
    def copy_from(cls, s):
        return cls(copy.deepcopy(s.env_params), copy.deepcopy(s.actor_critic), copy.deepcopy(s.agent),
                   copy.deepcopy(s.objs), s.optgraph_id)


def initial_sample(args, spec):
    """Warm-up policy + PPO + fresh env_params (morl/warm_up.py:33-68), without its evaluation."""
    policy = make_policy(spec['obs_dim'], spec['act_dim'], args.obj_num, layernorm=getattr(args, 'layernorm', False))
    agent = PPO(policy, args.clip_param, args.ppo_epoch, args.num_mini_batch, args.value_loss_coef,
                args.entropy_coef, lr=args.lr, eps=1e-5, max_grad_norm=args.max_grad_norm)
    env_params = {'ob_rms': RunningMeanStd(shape=(spec['obs_dim'],)) if args.ob_rms else None,
                  'ret_rms': RunningMeanStd(shape=()),
                  'obj_rms': RunningMeanStd(shape=()) if args.obj_rms else None}
    return OracleSample(env_params, policy, agent, optgraph_id=-1)


def evaluation(args, spec, s0_eval, policy, ob_rms):
    objs = np.zeros(args.obj_num)
    with torch.no_grad():
        for eval_id in range(args.eval_num):
            env = SynthEnv(spec, s0_eval[eval_id])
            ob = env.reset()
            done, gamma = False, 1.0
            while not done:
                if args.ob_rms:
                    ob = np.clip((ob - ob_rms.mean) / np.sqrt(ob_rms.var + 1e-8), -10.0, 10.0)
                _, action, _ = policy.act(torch.tensor(ob, dtype=next(policy.parameters()).dtype).unsqueeze(0),
                                          deterministic=True)
                ob, _, done, info = env.step(action[0].numpy())
                objs += gamma * info['obj']
                if not args.raw:
                    gamma *= args.gamma
    return objs / args.eval_num


def mopg_worker(args, spec, s0_train, s0_eval, sample, weights, iteration, num_updates,
                noise_fn=None, record=None):
    """Run num_updates PPO iterations of one task; returns the list of offspring OracleSamples.

    noise_fn(j) -> (noise [T,N,A] fp64 tensor, perms list[E]) replaces the RNG draws of
    iteration j; None reproduces the reference's own draws (torch.manual_seed(j)).
    record, if a list, receives per-iteration dicts of intermediate tensors.
    """
    sample = OracleSample.copy_from(sample)  # Task deep-copies its elite (morl/task.py:9-10)
    policy, agent = sample.actor_critic, sample.agent
    _to_net_dtype(policy, agent)
    T, N = args.num_steps, args.num_processes
    envs = VecNormalizedSynth(spec, s0_train, args.gamma, args.ob_rms, args.obj_rms)
    for key in ('ob_rms', 'ret_rms', 'obj_rms'):
        if sample.env_params.get(key) is not None:
            setattr(envs, key, sample.env_params[key].copy())
    ro = RolloutStorage(T, N, spec['obs_dim'], spec['act_dim'], args.obj_num)
    ro.obs[0].copy_(torch.from_numpy(envs.reset()).to(F64))
    total = int(args.num_env_steps) // T // N
    offspring = []
    for j in range(iteration, min(iteration + num_updates, total)):
        torch.manual_seed(j)
        noise, perms = noise_fn(j) if noise_fn is not None else (None, None)
        if args.use_linear_lr_decay:
            agent.set_lr(linear_lr(j, total, args.lr, args.lr_decay_ratio))
        for t in range(T):
            with torch.no_grad():
                value, action, logp = policy.act(ro.obs[t].to(NET), noise=None if noise is None else noise[t])
            obs, dones, infos = envs.step(action.numpy())
            obj = torch.tensor(np.stack([i['obj'] for i in infos]), dtype=F64)
            masks = torch.tensor([[0.0] if d else [1.0] for d in dones], dtype=F64)
            bad = torch.tensor([[0.0] if 'bad_transition' in i else [1.0] for i in infos], dtype=F64)
            ro.insert(torch.from_numpy(obs).to(F64), action, logp, value, obj, masks, bad)
        with torch.no_grad():
            next_value = policy.get_value(ro.obs[-1].to(NET))
        ro.compute_returns(next_value, args.use_gae, args.gamma, args.gae_lambda, args.use_proper_time_limits)
        obj_var = envs.obj_rms.var if envs.obj_rms is not None else None
        if record is not None:
            rec = {k: getattr(ro, k).clone() for k in ('obs', 'actions', 'action_log_probs', 'value_preds',
                                                         'rewards', 'masks', 'bad_masks', 'returns')}
            rec['obj_var'] = None if obj_var is None else np.array(obj_var, copy=True)
        stats = agent.update(ro, weights, obj_var, perms)
        ro.after_update()
        env_params = {k: (getattr(envs, k).copy() if getattr(envs, k) is not None else None)
                      for k in ('ob_rms', 'ret_rms', 'obj_rms')}
        snap = OracleSample(env_params, copy.deepcopy(policy), copy.deepcopy(agent))
        snap.objs = evaluation(args, spec, s0_eval, snap.actor_critic, env_params['ob_rms'])
        offspring.append(snap)
        if record is not None:
            rec['stats'] = stats
            rec['objs'] = snap.objs.copy()
            record.append(rec)
    return offspring
