"""Oracle: running statistics, synthetic MO env, and the vectorised env stack.

Restates (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py):
  * RunningMeanStd / Chan merge     -- externals/baselines/baselines/common/running_mean_std.py:3-31
  * VecNormalize.step_wait/_obfilt  -- externals/baselines/baselines/common/vec_env/vec_normalize.py:29-66
    (+ subclass _obfilt with training flag, a2c_ppo_acktr/envs.py:197-217)
  * DummyVecEnv auto-reset          -- externals/baselines/baselines/common/vec_env/dummy_vec_env.py:45-62
  * TimeLimit + TimeLimitMask       -- a2c_ppo_acktr/envs.py:122-131 (bad_transition at the time limit)
  * VecPyTorch obs cast to float32  -- a2c_ppo_acktr/envs.py:178-194

The MuJoCo physics is replaced by the build's synthetic env:
    a_c = clip(a, lo, hi);  s' = tanh(d*s + U a_c + c)
    obj = V s' + ebase - ecoef * sum(a_c^2)
fixed-length episodes (done only at the time limit, so bad_transition is always set).
"""
import numpy as np


class RunningMeanStd:
    """Parallel-variance running statistics (running_mean_std.py:3-31)."""

    def __init__(self, epsilon=1e-4, shape=()):
        self.mean = np.zeros(shape, 'float64')
        self.var = np.ones(shape, 'float64')
        self.count = epsilon

    def update(self, x):
        x = np.asarray(x, dtype=np.float64)
        self.update_from_moments(np.mean(x, axis=0), np.var(x, axis=0), x.shape[0])

    def update_from_moments(self, batch_mean, batch_var, batch_count):
        delta = batch_mean - self.mean
        tot = self.count + batch_count
        new_mean = self.mean + delta * batch_count / tot
        m2 = self.var * self.count + batch_var * batch_count + np.square(delta) * self.count * batch_count / tot
        self.mean, self.var, self.count = new_mean, m2 / tot, tot

    def copy(self):
        r = RunningMeanStd.__new__(RunningMeanStd)
        r.mean, r.var, r.count = np.array(self.mean, copy=True), np.array(self.var, copy=True), self.count
        return r


class SynthEnv:
    """One synthetic MO env instance (fp64, like MuJoCo state)."""

    def __init__(self, spec, s0):
        self.spec = spec
        self.s0 = np.asarray(s0, dtype=np.float64)
        self.s = None
        self.elapsed = 0

    def reset(self):
        self.s = self.s0.copy()
        self.elapsed = 0
        return self.s.copy()

    def step(self, a):
        sp = self.spec
        a_c = np.clip(np.asarray(a, dtype=np.float64), sp['act_lo'], sp['act_hi'])
        self.s = np.tanh(sp['d'] * self.s + sp['U'] @ a_c + sp['c'])
        obj = sp['V'] @ self.s + sp['ebase'] - sp['ecoef'] * np.sum(np.square(a_c))
        self.elapsed += 1
        done = self.elapsed >= sp['max_episode_steps']
        info = {'obj': obj}
        if done and self.elapsed == sp['max_episode_steps']:
            info['bad_transition'] = True  # TimeLimitMask (envs.py:125-126)
        return self.s.copy(), 0.0, done, info


class VecNormalizedSynth:
    """DummyVecEnv(N SynthEnv) + VecNormalize(ob=ob_rms, obj_rms) + VecPyTorch float32 cast."""

    def __init__(self, spec, s0_table, gamma, use_ob_rms=True, use_obj_rms=True, clipob=10., cliprew=10., epsilon=1e-8):
        self.envs = [SynthEnv(spec, s0) for s0 in s0_table]
        self.num_envs = len(self.envs)
        self.ob_rms = RunningMeanStd(shape=(spec['obs_dim'],)) if use_ob_rms else None
        self.ret_rms = RunningMeanStd(shape=())
        self.obj_rms = RunningMeanStd(shape=()) if use_obj_rms else None
        self.clipob, self.cliprew, self.gamma, self.epsilon = clipob, cliprew, gamma, epsilon
        self.ret = np.zeros(self.num_envs)
        self.obj = np.array([None] * self.num_envs)

    def _obfilt(self, obs):
        if self.ob_rms is None:
            return obs
        self.ob_rms.update(obs)
        return np.clip((obs - self.ob_rms.mean) / np.sqrt(self.ob_rms.var + self.epsilon), -self.clipob, self.clipob)

    def reset(self):
        self.ret = np.zeros(self.num_envs)
        obs = np.stack([e.reset() for e in self.envs])
        return self._obfilt(obs).astype(np.float32)

    def step(self, actions):
        """actions: [N, A] array. Returns (obs fp32 [N,O], dones [N], infos)."""
        obs_l, dones, infos = [], [], []
        for e, a in zip(self.envs, actions):
            o, r, d, info = e.step(a)
            if d:
                o = e.reset()
            obs_l.append(o)
            dones.append(d)
            infos.append(info)
        obs = np.stack(obs_l)
        dones = np.array(dones)
        rews = np.zeros(self.num_envs)
        self.ret = self.ret * self.gamma + rews
        for info in infos:
            info['obj_raw'] = info['obj']
        obj = np.array([info['obj'] for info in infos])
        self.obj = self.obj * self.gamma + obj if self.obj[0] is not None else obj
        obs = self._obfilt(obs)
        self.ret_rms.update(self.ret)
        if self.obj_rms is not None:
            self.obj_rms.update(self.obj)
            for info in infos:
                info['obj'] = np.clip(info['obj'] / np.sqrt(self.obj_rms.var + self.epsilon), -self.cliprew, self.cliprew)
        self.ret[dones] = 0.
        self.obj[dones] = np.zeros_like(self.obj[dones])
        return obs.astype(np.float32), dones, infos
