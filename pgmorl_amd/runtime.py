"""Device-resident state of P MOPG tasks on one GPU and the per-iteration kernel sequence.

One ``TaskBatch`` owns every HBM buffer of P tasks (parameters + Adam state, env state, running
statistics, rollout storage) and drives the libpgm kernels on torch's current stream:

    rollout (T steps, fused act + env + VecNormalize + insert + bootstrap value)
      -> gae -> adv_normalize -> ppo_update -> eval

i.e. one iteration of MOPG_worker's loop body (morl/mopg.py:95-155) for all tasks at once.
torch is used only for device memory and the stream; every op is a libpgm kernel and raises if
the library is unavailable (no CPU fallback).
"""
import ctypes as C
import math

import numpy as np
import torch

from . import envspec
from ._lib import (Dims, EnvSpec, EnvState, NormState, PGMError, PPOHParams, RolloutBuf, check, launch_opts, lib)
from .layout import ParamLayout

F32, F64, I32 = torch.float32, torch.float64, torch.int32
UPDATE_TIMEOUT_MSG = ('pgm_ppo_update: a cross-workgroup exchange timed out (workspace word 2P set); the update '
                      'kernel\'s workgroups were not co-resident -- the parameters are invalid')


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class TaskBatch:
    """HBM state of P tasks sharing env, rollout shape and PPO hyper-parameters.

    ``capacity`` (>= P) sizes every buffer once; ``set_active(P)`` then runs the first P task slots without
    reallocating (the generation loop keeps one TaskBatch for populations of varying size).  The public
    tensors (``params``, ``ob_mean``, ``obs``, ...) are views of the active slots.  Two packed regions make the
    per-iteration snapshot and the per-generation load single copies:
      * ``state``  [3][capacity][L] fp32: params | Adam exp_avg | exp_avg_sq (``params`` = state[0, :P], ...);
      * ``stats64`` flat fp64: the segments of ``STAT_SEGMENTS`` (task weights and every running statistic),
        each [capacity][width] contiguous -- a whole-buffer copy is one iteration's record of every task.
    """
    # (name, width per task: int, or the attribute of the dims it is); the order is the stats64 layout
    STAT_SEGMENTS = (('weights', 'K'), ('ob_mean', 'O'), ('ob_var', 'O'), ('ob_count', 0), ('ret_mean', 0),
                     ('ret_var', 0), ('ret_count', 0), ('obj_mean', 'K'), ('obj_var', 'K'), ('obj_count', 0))

    def __init__(self, env_name, P, num_processes=4, num_steps=2048, seed=0, eval_num=1, gamma=0.995,
                 gae_lambda=0.95, use_gae=True, use_proper_time_limits=True, ob_rms=True, obj_rms=True, raw=True,
                 clip_param=0.2, ppo_epoch=10, num_mini_batch=32, value_loss_coef=0.5, entropy_coef=0.0,
                 max_grad_norm=0.5, adam_eps=1e-5, use_clipped_value_loss=True, device='cuda', capacity=None):
        self.spec = envspec.make_spec(env_name)
        sp = self.spec
        self.env_name = env_name
        self.capacity = Pc = max(P, capacity or P)
        self.P, self.N, self.T = P, num_processes, num_steps
        self.O, self.A, self.K, self.H = sp['obs_dim'], sp['act_dim'], sp['obj_num'], 64
        self.eval_num, self.gamma, self.gae_lambda = eval_num, gamma, gae_lambda
        self.use_gae, self.proper = use_gae, use_proper_time_limits
        self.use_ob_rms, self.use_obj_rms, self.raw = ob_rms, obj_rms, raw
        self.ppo_epoch, self.num_mini_batch = ppo_epoch, num_mini_batch
        self.dev = torch.device(device)
        self.layout = ParamLayout(self.O, self.A, self.K, self.H)
        L, O, A, K, N, T = self.layout.total, self.O, self.A, self.K, self.N, self.T
        self._full = {}  # name -> full-capacity tensor whose leading dim is the task slot

        def z(name, *s, dt=F32, fill=0.0):
            t = torch.full((Pc,) + s, fill, dtype=dt, device=self.dev)
            self._full[name] = t
            return t
        # spec constants + reset tables (fp64)
        self._spec_t = {k: torch.tensor(np.ascontiguousarray(sp[k]), dtype=F64, device=self.dev)
                        for k in ('d', 'U', 'c', 'V', 'ebase', 'ecoef', 'act_lo', 'act_hi')}
        self.s0_train = torch.tensor(envspec.reset_table(O, seed, N), dtype=F64, device=self.dev)
        self.s0_eval = torch.tensor(envspec.reset_table(O, seed, eval_num), dtype=F64, device=self.dev)
        # policy + optimiser: one [3][Pc][L] region
        self._state = torch.zeros(3, Pc, L, dtype=F32, device=self.dev)
        z('adam_step', dt=I32)
        z('lr')
        # task weights + running statistics: one flat fp64 region (STAT_SEGMENTS)
        self._seg = []
        off = 0
        for name, wd in self.STAT_SEGMENTS:
            w = getattr(self, wd) if isinstance(wd, str) else 1
            self._seg.append((name, off, w, isinstance(wd, str)))
            off += Pc * w
        self._stats64 = torch.zeros(off, dtype=F64, device=self.dev)
        # env state
        z('s', N, O, dt=F64)
        z('elapsed', N, dt=I32)
        z('obj_acc', N, K, dt=F64)
        z('obj_valid', dt=I32)
        z('ret', N, dt=F64)
        # rollout storage (storage.py:12-30)
        z('obs', T + 1, N, O)
        z('actions', T, N, A)
        z('logp', T, N)
        z('values', T + 1, N, K)
        z('returns', T + 1, N, K)
        z('rewards', T, N, K)
        z('adv', T, N)
        z('masks', T + 1, N, fill=1.0)
        z('bad_masks', T + 1, N, fill=1.0)
        z('stats', 3)
        z('objs', K, dt=F64)
        # the overlapped evaluation's copy of ob_rms: mean | var of every slot, one copy of the adjacent stats64
        # segments ob_mean, ob_var (STAT_SEGMENTS order)
        self._eval_ob = torch.zeros(2, Pc, O, dtype=F64, device=self.dev)
        self.perms = torch.zeros(ppo_epoch, T * N, dtype=I32, device=self.dev)
        self.noise = torch.zeros(T, N, A, dtype=F32, device=self.dev)
        self.hp = PPOHParams(clip_param=clip_param, value_loss_coef=value_loss_coef, entropy_coef=entropy_coef,
                             max_grad_norm=max_grad_norm, adam_eps=adam_eps, beta1=0.9, beta2=0.999,
                             ppo_epoch=ppo_epoch, num_mini_batch=num_mini_batch,
                             use_clipped_value_loss=int(use_clipped_value_loss))
        self._eval_stream, self._eval_done = None, None
        self._reset_pending = False  # a pgm_ppo_update_reset queued on the side stream, not yet waited for
        nws = lib().pgm_ppo_update_workspace_bytes(C.byref(Dims(Pc, N, T, O, A, K, self.H)))
        self.update_ws = torch.zeros((nws + 7) // 8, dtype=torch.int64, device=self.dev)
        # sticky OR of every update's exchange-timeout word (workspace word 2P, include/pgm_abi.h): a launch
        # whose spin-wait gave up produced invalid parameters; check_update() turns that into PGMError
        self.update_failed = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.last_fail_word = 0
        self.set_active(P)
        self.reset_stats()

    def set_active(self, P):
        """Run the first P task slots (P <= capacity): re-slices the public views and the kernels' dims."""
        if not 0 < P <= self.capacity:
            raise ValueError(f'active tasks {P} outside [1, capacity {self.capacity}]')
        self.P = P
        for name, t in self._full.items():
            setattr(self, name, t[:P])
        self.params, self.adam_m, self.adam_v = self._state[0, :P], self._state[1, :P], self._state[2, :P]
        for name, off, w, vec in self._seg:
            v = self._stats64[off:off + self.capacity * w]
            setattr(self, name, (v.view(self.capacity, w) if vec else v)[:P])
            if name == 'ob_mean':
                self._ob_src = self._stats64[off:off + 2 * self.capacity * w].view(2, self.capacity, w)
        self._eval_mean, self._eval_var = self._eval_ob[0, :P], self._eval_ob[1, :P]
        self._build_structs()

    @property
    def state(self):
        """[3][P][L] view of the active slots (params | exp_avg | exp_avg_sq); strided when P < capacity."""
        return self._state[:, :self.P]

    def stats64_record(self, out):
        """Copy the whole flat fp64 statistics region (weights + every running statistic of every slot) into
        ``out`` (one device copy: an iteration's snapshot record, unpacked on the host by stat_views)."""
        out.copy_(self._stats64)

    def stat_views(self, flat, P=None):
        """Host-side split of a stats64 record (numpy [n]) into {name: [P, width] or [P]} arrays."""
        P = self.P if P is None else P
        out = {}
        for name, off, w, vec in self._seg:
            v = flat[off:off + self.capacity * w]
            out[name] = (v.reshape(self.capacity, w) if vec else v)[:P]
        return out

    def load_stats64(self, host_flat):
        """One H2D copy of a host-built stats64 image (numpy fp64, the stat_views layout)."""
        self._stats64.copy_(torch.from_numpy(np.ascontiguousarray(host_flat, dtype=np.float64)))

    def new_stats64(self):
        """A host stats64 image holding fresh RunningMeanStd values (count 1e-4, mean 0, var 1) and zero weights."""
        flat = np.zeros(self._stats64.numel(), dtype=np.float64)
        v = self.stat_views(flat, self.capacity)
        for var in (v['ob_var'], v['ret_var'], v['obj_var']):
            var[...] = 1.0
        for cnt in (v['ob_count'], v['ret_count'], v['obj_count']):
            cnt[...] = 1e-4
        return flat

    # ------------------------------------------------------------------ structs
    def _build_structs(self):
        self.dims = Dims(self.P, self.N, self.T, self.O, self.A, self.K, self.H)
        st = self._spec_t
        self.c_spec = EnvSpec(_ptr(st['d']), _ptr(st['U']), _ptr(st['c']), _ptr(st['V']), _ptr(st['ebase']),
                              _ptr(st['ecoef']), _ptr(st['act_lo']), _ptr(st['act_hi']),
                              self.spec['max_episode_steps'], 0)
        self.c_state = EnvState(_ptr(self.s), _ptr(self.elapsed), _ptr(self.obj_acc), _ptr(self.obj_valid),
                                _ptr(self.ret), _ptr(self.s0_train))
        self.c_norm = NormState(_ptr(self.ob_mean), _ptr(self.ob_var), _ptr(self.ob_count), _ptr(self.ret_mean),
                                _ptr(self.ret_var), _ptr(self.ret_count), _ptr(self.obj_mean), _ptr(self.obj_var),
                                _ptr(self.obj_count), self.gamma, 10.0, 10.0, 1e-8, int(self.use_ob_rms),
                                int(self.use_obj_rms))
        self.c_rb = RolloutBuf(*(_ptr(t) for t in (self.obs, self.actions, self.logp, self.values, self.rewards,
                                                   self.masks, self.bad_masks, self.returns, self.adv)))

    def reset_stats(self):
        """Fresh RunningMeanStd objects: count 1e-4, mean 0, var 1 (running_mean_std.py:5-8)."""
        for mean, var, cnt in ((self.ob_mean, self.ob_var, self.ob_count), (self.ret_mean, self.ret_var, self.ret_count),
                               (self.obj_mean, self.obj_var, self.obj_count)):
            mean.zero_()
            var.fill_(1.0)
            cnt.fill_(1e-4)

    # ------------------------------------------------------------------ kernels
    def env_reset(self):
        """Fresh make_vec_envs + envs.reset() (mopg.py:67-82): obs[:, 0], masks[:, 0] = 1."""
        out = torch.empty(self.P, self.N, self.O, dtype=F32, device=self.dev)
        check(lib().pgm_env_reset(C.byref(self.dims), C.byref(self.c_spec), C.byref(self.c_state),
                                  C.byref(self.c_norm), _ptr(out), _stream()), 'pgm_env_reset')
        self.obs[:, 0].copy_(out)
        self.masks[:, 0] = 1.0
        self.bad_masks[:, 0] = 1.0
        return out

    def env_step(self, action):
        P, N, O, K = self.P, self.N, self.O, self.K
        action = action.to(device=self.dev, dtype=F32).contiguous()
        obs = torch.empty(P, N, O, dtype=F32, device=self.dev)
        rew = torch.empty(P, N, K, dtype=F32, device=self.dev)
        m, b = torch.empty(P, N, dtype=F32, device=self.dev), torch.empty(P, N, dtype=F32, device=self.dev)
        check(lib().pgm_env_step(C.byref(self.dims), C.byref(self.c_spec), C.byref(self.c_state),
                                 C.byref(self.c_norm), _ptr(action), _ptr(obs), _ptr(rew), _ptr(m), _ptr(b),
                                 _stream()), 'pgm_env_step')
        return obs, rew, m, b

    def act(self, obs, noise=None, deterministic=False):
        P, N = self.P, obs.shape[1]
        obs = obs.to(device=self.dev, dtype=F32).contiguous()
        d = Dims(P, N, self.T, self.O, self.A, self.K, self.H)
        value = torch.empty(P, N, self.K, dtype=F32, device=self.dev)
        action = torch.empty(P, N, self.A, dtype=F32, device=self.dev)
        logp = torch.empty(P, N, dtype=F32, device=self.dev)
        nz = None if noise is None else noise.to(device=self.dev, dtype=F32).contiguous()
        check(lib().pgm_act_forward(C.byref(d), _ptr(self.params), _ptr(obs), _ptr(nz), int(deterministic),
                                    _ptr(value), _ptr(action), _ptr(logp), _stream()), 'pgm_act_forward')
        return value, action, logp

    def rollout(self, seed, noise=None, carry=True):
        nz = None
        if noise is not None:
            if noise is not self.noise:
                self.noise.copy_(noise.to(dtype=F32))
            nz = self.noise
        check(lib().pgm_rollout(C.byref(self.dims), _ptr(self.params), C.byref(self.c_spec), C.byref(self.c_state),
                                C.byref(self.c_norm), C.byref(self.c_rb), _ptr(nz), C.c_uint64(seed),
                                int(carry), C.byref(launch_opts()), _stream()), 'pgm_rollout')

    def gae(self):
        check(lib().pgm_gae(C.byref(self.dims), C.byref(self.c_rb), self.gamma, self.gae_lambda, int(self.use_gae),
                            int(self.proper), _stream()), 'pgm_gae')

    def adv_normalize(self):
        var = self.obj_var if self.use_obj_rms else None
        check(lib().pgm_adv_normalize(C.byref(self.dims), C.byref(self.c_rb), _ptr(self.weights), _ptr(var),
                                      _stream()), 'pgm_adv_normalize')

    def make_perms(self, seed):
        E, n = self.perms.shape
        check(lib().pgm_randperm(n, E, C.c_uint64(seed), _ptr(self.perms), _stream()), 'pgm_randperm')

    def ppo_update(self, perms=None, defer_flag=False):
        """The update on the current stream.  The exchange-timeout word of this launch is OR-ed into the sticky
        ``update_failed`` flag on the current stream, or (defer_flag) left to ``fold_update_flag`` on a stream that
        runs before the next update's launch (which resets the word)."""
        if self._reset_pending:  # the workspace reset queued on the side stream must land first
            self.wait_eval()
        if perms is not None:
            self.perms.copy_(torch.as_tensor(np.asarray(perms), dtype=I32))
        self.ppo_update_launch()
        if not defer_flag:
            self.fold_update_flag()

    def fold_update_flag(self):
        flag = self.update_ws[2 * self.P:2 * self.P + 1]
        torch.bitwise_or(self.update_failed, flag, out=self.update_failed)  # stream-ordered, no host sync

    def ppo_update_launch(self):
        """pgm_ppo_update alone (packed rows + the update kernel) on the current stream."""
        check(lib().pgm_ppo_update(C.byref(self.dims), C.byref(self.hp), _ptr(self.params), _ptr(self.adam_m),
                                   _ptr(self.adam_v), _ptr(self.adam_step), _ptr(self.lr), _ptr(self.perms),
                                   C.byref(self.c_rb), _ptr(self.stats), _ptr(self.update_ws),
                                   C.byref(launch_opts()), _stream()), 'pgm_ppo_update')

    def update_variant(self):
        """The update kernel pgm_ppo_update launches for this batch (pgm_ppo_update_variant: the launcher's own rule)."""
        buf = C.create_string_buffer(128)
        check(lib().pgm_ppo_update_variant(C.byref(self.dims), C.byref(self.hp), C.byref(launch_opts()), buf, 128),
              'pgm_ppo_update_variant')
        return buf.value.decode()

    def take_update_failed(self):
        """True if any PPO update since the last call timed out in a cross-workgroup exchange (its parameters /
        Adam state are invalid); resets the sticky flag.  Synchronises with the stream (after the overlapped
        evaluation, whose stream folds the last update's flag)."""
        self.wait_eval()
        word = int(self.update_failed.item())
        self.last_fail_word = word  # (the OR of the timed-out launches' words: kernels may encode the wait site)
        if word != 0:
            self.update_failed.zero_()
        return word != 0

    def check_update(self):
        """Raise PGMError if any PPO update since the last check timed out (take_update_failed).  Call it once
        per generation or after a timed region, not per update.  Multi-GPU callers share the flag across ranks
        first (MOPGPopulation.run) so that every rank raises together."""
        if self.take_update_failed():
            raise PGMError(f'{UPDATE_TIMEOUT_MSG} (word 0x{self.last_fail_word & (2**64 - 1):x})')

    def evaluate(self, ob_mean=None, ob_var=None, out=None):
        mean = self.ob_mean if ob_mean is None else ob_mean
        var = self.ob_var if ob_var is None else ob_var
        out = self.objs if out is None else out
        check(lib().pgm_eval(C.byref(self.dims), _ptr(self.params), C.byref(self.c_spec), _ptr(mean), _ptr(var),
                             _ptr(self.s0_eval), self.eval_num, int(self.use_ob_rms), int(self.raw), self.gamma,
                             _ptr(out), C.byref(launch_opts()), _stream()), 'pgm_eval')
        return out

    @property
    def eval_stream(self):
        """Side stream of the overlapped evaluation (iteration(..., overlap_eval=True))."""
        if self._eval_stream is None:
            self._eval_stream = torch.cuda.Stream(device=self.dev)
        return self._eval_stream

    def wait_eval(self):
        """Order the current stream after the last overlapped evaluation (its objs are then readable)."""
        if self._eval_done is not None:
            torch.cuda.current_stream().wait_event(self._eval_done)
        self._reset_pending = False

    def iteration(self, j, lr, noise=None, perms=None, carry=True, overlap_eval=False, objs_out=None):
        """One MOPG iteration for every task: rollout, returns, advantages, PPO update, evaluation.

        noise/perms: the reference's RNG draws of iteration j (parity mode); None draws the
        device counter streams keyed by j (perf mode).

        overlap_eval: the evaluation of this iteration's snapshot (mopg.py:146-155) runs on a side stream,
        concurrently with the NEXT iteration's rollout / returns / advantages (which only read the
        parameters); the next PPO update (which writes them) waits for it.  It normalises with a copy of
        this iteration's ob_rms (the next rollout advances the live one) and writes objs_out (default
        self.objs), readable after wait_eval() or from work queued on eval_stream."""
        if noise is None:  # perf mode: the counter stream of iteration j, drawn by one wide kernel up front
            check(lib().pgm_normal_noise(self.noise.numel(), C.c_uint64(j), _ptr(self.noise), _stream()),
                  'pgm_normal_noise')
            noise = self.noise
        perm_ready = None
        if perms is None and overlap_eval:  # the permutations (and lr) only feed the update: set beside the rollout
            side = self.eval_stream  # (behind the previous evaluation, itself behind the previous update)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                self.lr.fill_(float(lr))
                self.make_perms(j)
                perm_ready = torch.cuda.Event()
                perm_ready.record(side)
        else:
            self.lr.fill_(float(lr))
        self.rollout(j, noise=noise, carry=carry)
        self.gae()
        self.adv_normalize()
        if perm_ready is not None:
            # one wait: the side stream ran the previous evaluation (which still reads the parameters) and the
            # workspace reset first
            torch.cuda.current_stream().wait_event(perm_ready)
            self._reset_pending = False
        else:
            if perms is None:
                self.make_perms(j)
            self.wait_eval()  # the previous overlapped evaluation still reads the parameters
        self.ppo_update(perms, defer_flag=overlap_eval)
        if not overlap_eval:
            self.evaluate(out=objs_out)
            return
        if self.P == self.capacity:
            self._eval_ob.copy_(self._ob_src)  # ob_mean | ob_var in one copy
        else:
            self._eval_mean.copy_(self.ob_mean)
            self._eval_var.copy_(self.ob_var)
        ready = torch.cuda.Event()
        ready.record()
        side = self.eval_stream
        side.wait_event(ready)
        with torch.cuda.stream(side):
            # the timeout word of this update, folded off the main stream, then the next update's workspace reset
            # (the next update waits for this stream: perm_ready)
            self.fold_update_flag()
            check(lib().pgm_ppo_update_reset(C.byref(self.dims), _ptr(self.update_ws), _stream()),
                  'pgm_ppo_update_reset')
            self._reset_pending = True
            out = self.evaluate(self._eval_mean, self._eval_var, out=objs_out)
            out.record_stream(side)
            self._eval_done = torch.cuda.Event()
            self._eval_done.record(side)

    # ------------------------------------------------------------------ host transfer
    def set_task(self, p, state_dict, opt_state=None, env_params=None, weights=None):
        lay = self.layout
        self.params[p].copy_(torch.from_numpy(lay.flatten(state_dict)))
        m, v, step = lay.adam_from_optimizer_state(opt_state or {})
        self.adam_m[p].copy_(torch.from_numpy(m))
        self.adam_v[p].copy_(torch.from_numpy(v))
        self.adam_step[p] = step
        if weights is not None:
            self.weights[p].copy_(torch.as_tensor(np.asarray(weights, dtype=np.float64)))
        if env_params is not None:
            self.set_env_params(p, env_params)

    def set_env_params(self, p, env_params):
        """Restore ob_rms / ret_rms / obj_rms (mopg.py:70-75); obj_rms may still be scalar-shaped."""
        K = self.K
        ob, rt, oj = env_params.get('ob_rms'), env_params.get('ret_rms'), env_params.get('obj_rms')
        if ob is not None:
            self.ob_mean[p].copy_(torch.as_tensor(np.asarray(ob.mean, np.float64)))
            self.ob_var[p].copy_(torch.as_tensor(np.asarray(ob.var, np.float64)))
            self.ob_count[p] = float(ob.count)
        if rt is not None:
            self.ret_mean[p] = float(np.asarray(rt.mean).reshape(-1)[0])
            self.ret_var[p] = float(np.asarray(rt.var).reshape(-1)[0])
            self.ret_count[p] = float(rt.count)
        if oj is not None:
            self.obj_mean[p].copy_(torch.as_tensor(np.broadcast_to(np.asarray(oj.mean, np.float64), (K,)).copy()))
            self.obj_var[p].copy_(torch.as_tensor(np.broadcast_to(np.asarray(oj.var, np.float64), (K,)).copy()))
            self.obj_count[p] = float(oj.count)

    def get_params(self, p):
        return self.layout.unflatten(self.params[p])
