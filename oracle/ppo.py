"""Oracle: rollout storage, vector GAE and the scalarised PPO update (torch CPU, fp64).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates:
  * RolloutStorage (buffers, insert, after_update)        -- a2c_ppo_acktr/storage.py:9-75
  * compute_returns (4 variants: gae x proper_time_limits) -- a2c_ppo_acktr/storage.py:77-116
  * feed_forward_generator (SubsetRandomSampler + BatchSampler(drop_last=True))
                                                          -- a2c_ppo_acktr/storage.py:118-154
  * PPO.update (un-normalise returns by sqrt(obj_var+1e-8), weighted-sum scalarise,
    unbiased-std advantage normalisation, clipped surrogate + clipped value loss,
    clip_grad_norm_, Adam)                                -- a2c_ppo_acktr/algo/ppo.py:7-115
  * WeightedSumScalarization.evaluate                     -- morl/scalarization_methods.py:21-29
  * update_linear_schedule                                -- a2c_ppo_acktr/utils.py:46-50
"""
import numpy as np
import torch
import torch.nn as nn
import torch.optim as optim

F64 = torch.float64


class RolloutStorage:
    def __init__(self, T, N, obs_dim, act_dim, obj_num):
        self.obs = torch.zeros(T + 1, N, obs_dim, dtype=F64)
        self.rewards = torch.zeros(T, N, obj_num, dtype=F64)
        self.value_preds = torch.zeros(T + 1, N, obj_num, dtype=F64)
        self.returns = torch.zeros(T + 1, N, obj_num, dtype=F64)
        self.action_log_probs = torch.zeros(T, N, 1, dtype=F64)
        self.actions = torch.zeros(T, N, act_dim, dtype=F64)
        self.masks = torch.ones(T + 1, N, 1, dtype=F64)
        self.bad_masks = torch.ones(T + 1, N, 1, dtype=F64)
        self.num_steps = T
        self.step = 0

    def insert(self, obs, actions, logp, values, rewards, masks, bad_masks):
        s = self.step
        self.obs[s + 1].copy_(obs)
        self.actions[s].copy_(actions)
        self.action_log_probs[s].copy_(logp)
        self.value_preds[s].copy_(values)
        self.rewards[s].copy_(rewards)
        self.masks[s + 1].copy_(masks)
        self.bad_masks[s + 1].copy_(bad_masks)
        self.step = (s + 1) % self.num_steps

    def after_update(self):
        self.obs[0].copy_(self.obs[-1])
        self.masks[0].copy_(self.masks[-1])
        self.bad_masks[0].copy_(self.bad_masks[-1])

    def compute_returns(self, next_value, use_gae, gamma, lam, use_proper_time_limits=True):
        compute_returns_inplace(self.rewards, self.value_preds, self.masks, self.bad_masks, self.returns,
                                next_value, use_gae, gamma, lam, use_proper_time_limits)

    def minibatches(self, advantages, num_mini_batch, perm):
        """Yields the feed_forward_generator tuples for one epoch given that epoch's permutation."""
        T, N = self.rewards.shape[0:2]
        B = T * N
        mb = B // num_mini_batch
        flat = lambda x: x.reshape(B, *x.shape[2:])
        obs, act = flat(self.obs[:-1]), flat(self.actions)
        vp, ret = flat(self.value_preds[:-1]), flat(self.returns[:-1])
        lp, adv = flat(self.action_log_probs), advantages.reshape(B, 1)
        for b in range(B // mb):
            idx = perm[b * mb:(b + 1) * mb]
            yield obs[idx], act[idx], vp[idx], ret[idx], lp[idx], adv[idx]


def compute_returns_inplace(rewards, value_preds, masks, bad_masks, returns, next_value,
                            use_gae, gamma, lam, use_proper_time_limits):
    """Reverse sweep of storage.py:83-116 (in place on returns / value_preds[-1])."""
    T = rewards.shape[0]
    if use_gae:
        value_preds[-1] = next_value
        gae = 0
        for t in reversed(range(T)):
            delta = rewards[t] + gamma * value_preds[t + 1] * masks[t + 1] - value_preds[t]
            gae = delta + gamma * lam * masks[t + 1] * gae
            if use_proper_time_limits:
                gae = gae * bad_masks[t + 1]
            returns[t] = gae + value_preds[t]
    else:
        returns[-1] = next_value
        for t in reversed(range(T)):
            if use_proper_time_limits:
                returns[t] = (returns[t + 1] * gamma * masks[t + 1] + rewards[t]) * bad_masks[t + 1] \
                    + (1 - bad_masks[t + 1]) * value_preds[t]
            else:
                returns[t] = returns[t + 1] * gamma * masks[t + 1] + rewards[t]


def scalarized_normalized_advantages(returns, value_preds, weights, obj_var):
    """ppo.py:41-56: advantages [T,N] (normalised, unbiased std) from [T+1,N,K] returns/values."""
    if obj_var is not None:
        scale = torch.tensor(np.sqrt(np.asarray(obj_var, dtype=np.float64) + 1e-8), dtype=F64)
        returns = returns * scale
        value_preds = value_preds * scale
    w = torch.as_tensor(np.asarray(weights, dtype=np.float64))
    adv = (returns[:-1] * w).sum(-1) - (value_preds[:-1] * w).sum(-1)
    axis = tuple(range(adv.dim()))
    return (adv - adv.mean(axis=axis)) / (adv.std(axis=axis) + 1e-5)


def randperms(ppo_epoch, batch_size):
    """The RNG draws of one PPO.update: one randperm per epoch (SubsetRandomSampler)."""
    return [torch.randperm(batch_size) for _ in range(ppo_epoch)]


class PPO:
    def __init__(self, actor_critic, clip_param=0.2, ppo_epoch=10, num_mini_batch=32, value_loss_coef=0.5,
                 entropy_coef=0.0, lr=3e-4, eps=1e-5, max_grad_norm=0.5, use_clipped_value_loss=True):
        self.actor_critic = actor_critic
        self.clip_param, self.ppo_epoch, self.num_mini_batch = clip_param, ppo_epoch, num_mini_batch
        self.value_loss_coef, self.entropy_coef = value_loss_coef, entropy_coef
        self.max_grad_norm, self.use_clipped_value_loss = max_grad_norm, use_clipped_value_loss
        self.optimizer = optim.Adam(actor_critic.parameters(), lr=lr, eps=eps)

    def set_lr(self, lr):
        for g in self.optimizer.param_groups:
            g['lr'] = lr

    def minibatch_step(self, obs, act, vp, ret, old_lp, adv):
        """One clipped-PPO Adam step (ppo.py:76-103). Returns (value_loss, action_loss, entropy)."""
        dt = next(self.actor_critic.parameters()).dtype  # fp64; fp32 in the precision arm (oracle/mopg.py NET)
        if dt != F64:
            obs, act, vp, ret, old_lp, adv = (x.to(dt) for x in (obs, act, vp, ret, old_lp, adv))
        values, logp, entropy = self.actor_critic.evaluate_actions(obs, act)
        ratio = torch.exp(logp - old_lp)
        surr1 = ratio * adv
        surr2 = torch.clamp(ratio, 1.0 - self.clip_param, 1.0 + self.clip_param) * adv
        action_loss = -torch.min(surr1, surr2).mean()
        if self.use_clipped_value_loss:
            v_clip = vp + (values - vp).clamp(-self.clip_param, self.clip_param)
            value_loss = 0.5 * torch.max((values - ret).pow(2), (v_clip - ret).pow(2)).mean()
        else:
            value_loss = 0.5 * (ret - values).pow(2).mean()
        self.optimizer.zero_grad()
        (value_loss * self.value_loss_coef + action_loss - entropy * self.entropy_coef).backward()
        nn.utils.clip_grad_norm_(self.actor_critic.parameters(), self.max_grad_norm)
        self.optimizer.step()
        return value_loss.item(), action_loss.item(), entropy.item()

    def update(self, rollouts, weights, obj_var, perms=None):
        """PPO.update(rollouts, scalarization, obj_var) with optional explicit per-epoch permutations."""
        adv = scalarized_normalized_advantages(rollouts.returns, rollouts.value_preds, weights, obj_var)
        B = rollouts.rewards.shape[0] * rollouts.rewards.shape[1]
        vl = al = de = 0.0
        for e in range(self.ppo_epoch):
            perm = perms[e] if perms is not None else torch.randperm(B)
            for mbt in rollouts.minibatches(adv, self.num_mini_batch, perm):
                a, b, c = self.minibatch_step(*mbt)
                vl, al, de = vl + a, al + b, de + c
        n = self.ppo_epoch * self.num_mini_batch
        return vl / n, al / n, de / n


def linear_lr(j, total_num_updates, lr, lr_decay_ratio=1.0):
    epoch = j * lr_decay_ratio
    return lr - (lr * (epoch / float(total_num_updates)))
