"""MOPGPopulation: the drop-in replacement of the per-task process fan-out of one generation.

Reference: morl/morl.py:79-99 forks one ``MOPG_worker`` process per task (morl/mopg.py:60-182) and
gathers ``{'task_id', 'offspring_batch', 'done'}`` dicts from a multiprocessing Queue.  Here every
task of the generation lives in one ``TaskBatch`` on the GPU and each PPO iteration of all tasks
is a short sequence of libpgm kernels; ``run`` returns the same ``all_offspring_batch`` structure
(list over tasks of the per-iteration offspring Samples), so the rest of the generation loop is
unchanged.

RNG: ``rng='host'`` draws exactly what the reference draws for iteration j (torch.manual_seed(j),
then T Normal samples of shape [N, A] and ppo_epoch randperms of T*N, morl/mopg.py:96 and
storage.py:133) and uploads them -- bit-compatible with the CPU oracle; ``rng='device'`` uses the
counter-based device streams keyed by j (same distribution, no host work; the benchmark mode).
Like the reference, all tasks of an iteration share one noise stream.
"""
import os
import time

import numpy as np
import torch

from .runtime import TaskBatch
from .sample import DeviceSnapshot, RowStore, RunningMeanStd, Sample
from .shard import allgather_rows, move_rows, owner_of, task_block, world


def host_draws(j, T, N, A, E):
    torch.manual_seed(j)
    z = torch.stack([torch.normal(torch.zeros(N, A, dtype=torch.float64), torch.ones(N, A, dtype=torch.float64))
                     for _ in range(T)])
    perms = torch.stack([torch.randperm(T * N) for _ in range(E)])
    return z.float(), perms.to(torch.int32)


def linear_lr(j, total_num_updates, lr, ratio=1.0):
    """update_linear_schedule (a2c_ppo_acktr/utils.py:46-50) as called at morl/mopg.py:97-101."""
    return lr - lr * (j * ratio / float(total_num_updates))


class MOPGPopulation:
    def __init__(self, args, device='cuda', rng='device'):
        self.args = args
        self.device = torch.device(device)
        self.rng = rng
        self.tb = None
        self.moved_bytes = 0  # snapshot bytes this rank contributed to move_rows (multi-GPU)

    @property
    def layout(self):
        """The flat parameter layout of this run's env dims (pgm_param_layout)."""
        from .envspec import make_spec
        from .layout import ParamLayout
        if self.tb is not None:
            return self.tb.layout
        spec = make_spec(self.args.env_name)
        return ParamLayout(spec['obs_dim'], spec['act_dim'], spec['obj_num'])

    def _batch(self, P):
        """The one TaskBatch of this runtime, P active task slots.  Allocated once (re-allocated only when a
        generation needs more slots than any before): populations of varying size reuse its buffers."""
        a = self.args
        if self.tb is None or self.tb.capacity < P:
            cap = max(P, getattr(a, 'num_tasks', 0) or 0) if self.tb is None else P
            rank, ws = world()
            cap = min(cap, max(P, -(-cap // ws)))  # a rank only ever holds its block of the population
            self.tb = TaskBatch(a.env_name, P, num_processes=a.num_processes, num_steps=a.num_steps, seed=a.seed,
                                eval_num=a.eval_num, gamma=a.gamma, gae_lambda=a.gae_lambda, use_gae=a.use_gae,
                                use_proper_time_limits=a.use_proper_time_limits, ob_rms=a.ob_rms,
                                obj_rms=a.obj_rms, raw=a.raw, clip_param=a.clip_param, ppo_epoch=a.ppo_epoch,
                                num_mini_batch=a.num_mini_batch, value_loss_coef=a.value_loss_coef,
                                entropy_coef=a.entropy_coef, max_grad_norm=a.max_grad_norm, device=self.device,
                                capacity=cap)
        else:
            self.tb.set_active(P)
        return self.tb

    def load_tasks(self, tb, samples, weights):
        """Restore every active slot from its elite (mopg.py:67-82 per task, here batched): parameters + Adam
        moments by one gather of the snapshots' [3, L] blocks, the running statistics and task weights by one
        H2D copy of a host-built stats64 image, the Adam steps by one small copy."""
        P = len(samples)
        tb.set_active(P)
        blocks = [s.snapshot.block() for s in samples]
        tb.state.copy_(torch.stack(blocks, dim=1))
        flat = tb.new_stats64()
        v = tb.stat_views(flat, P)
        K = tb.K
        for p, (s, w) in enumerate(zip(samples, weights)):
            v['weights'][p] = np.asarray(w, dtype=np.float64)
            ep = s.env_params or {}
            ob, rt, oj = ep.get('ob_rms'), ep.get('ret_rms'), ep.get('obj_rms')
            if ob is not None:
                v['ob_mean'][p], v['ob_var'][p], v['ob_count'][p] = ob.mean, ob.var, float(ob.count)
            if rt is not None:
                v['ret_mean'][p] = float(np.asarray(rt.mean).reshape(-1)[0])
                v['ret_var'][p] = float(np.asarray(rt.var).reshape(-1)[0])
                v['ret_count'][p] = float(rt.count)
            if oj is not None:  # obj_rms may still be scalar-shaped (vec_normalize.py:21)
                v['obj_mean'][p] = np.broadcast_to(np.asarray(oj.mean, np.float64), (K,))
                v['obj_var'][p] = np.broadcast_to(np.asarray(oj.var, np.float64), (K,))
                v['obj_count'][p] = float(oj.count)
        tb.load_stats64(flat)
        tb.adam_step.copy_(torch.tensor([s.snapshot.adam_step for s in samples], dtype=torch.int32))

    def load_task(self, tb, p, sample, weights):
        """One slot (tests / tools); the generation loop uses load_tasks."""
        snap = sample.snapshot
        tb.params[p].copy_(snap.params)
        tb.adam_m[p].copy_(snap.adam_m)
        tb.adam_v[p].copy_(snap.adam_v)
        tb.adam_step[p] = snap.adam_step
        tb.weights[p].copy_(torch.as_tensor(np.asarray(weights, dtype=np.float64)))
        ep = sample.env_params or {}
        tb.set_env_params(p, {k: v for k, v in ep.items() if v is not None})

    def _env_params(self, st, p, O, K):
        """Slot p of a host stats64 record (TaskBatch.stat_views) -> env_params RunningMeanStd copies."""
        ep = {'ob_rms': None, 'ret_rms': None, 'obj_rms': None}
        if self.args.ob_rms:
            r = RunningMeanStd(shape=(O,))
            r.mean, r.var, r.count = st['ob_mean'][p].copy(), st['ob_var'][p].copy(), float(st['ob_count'][p])
            ep['ob_rms'] = r
        r = RunningMeanStd(shape=())
        r.mean, r.var, r.count = np.float64(st['ret_mean'][p]), np.float64(st['ret_var'][p]), float(st['ret_count'][p])
        ep['ret_rms'] = r
        if self.args.obj_rms:
            r = RunningMeanStd(shape=())
            r.mean, r.var, r.count = st['obj_mean'][p].copy(), st['obj_var'][p].copy(), float(st['obj_count'][p])
            ep['obj_rms'] = r
        return ep

    def place(self, samples, dsts):
        """Collective (every rank, same arguments): move each sample's snapshot to rank dsts[k] when it lives
        elsewhere (shard.move_rows).  A no-op in one process."""
        rank, ws = world()
        if ws == 1:
            return 0
        snaps = [s.snapshot for s in samples]
        moves = [(sn.owner if sn.owner is not None else -1, d) for sn, d in zip(snaps, dsts)]
        local = {k: snaps[k].stacked() for k, (src, _) in enumerate(moves) if src == rank}
        L = self.layout.total
        got, nbytes = move_rows(moves, local, (3, L), torch.float32, self.device)
        for k, rows in got.items():  # owner metadata stays as it is on every rank (identical move lists)
            snaps[k].adopt(rows)
        self.moved_bytes += nbytes
        return nbytes

    def materialize(self, samples, dst=0):
        """Collective: gather the snapshots of ``samples`` onto rank ``dst`` (final/EP_policy_*.pt)."""
        return self.place(samples, [dst] * len(samples))

    def check_generation(self, tb, step_mismatch=None):
        """Collective (every rank, also one without tasks): PGMError on EVERY rank when any rank's update timed
        out in a cross-workgroup exchange this generation, and RuntimeError on every rank when any rank's Adam
        step counts are not the expected ones (``step_mismatch``: that rank's message), before anyone enters the
        record all-gather (a rank raising alone would leave the others blocked in that collective)."""
        from ._lib import PGMError
        from .runtime import UPDATE_TIMEOUT_MSG
        from .shard import allreduce_max
        failed = bool(tb.take_update_failed()) if tb is not None else False
        rank, ws = world()
        any_failed, any_mismatch = (allreduce_max([float(failed), float(step_mismatch is not None)], self.device)
                                    if ws > 1 else (float(failed), float(step_mismatch is not None)))
        if any_failed:
            raise PGMError(UPDATE_TIMEOUT_MSG + ('' if failed else ' (on another rank)'))
        if any_mismatch:
            raise RuntimeError(step_mismatch or 'Adam step counts differ from the expected ones on another rank')

    def run(self, task_batch, iteration, num_updates, start_time=None, log=print):
        """Every task's MOPG iterations [iteration, iteration + num_updates) -> all_offspring_batch.

        Per iteration the device state of all local tasks is snapshotted by ONE copy into this generation's
        arena ([I][3][Pl][L]) and the running statistics by ONE copy of the stats64 region; the offspring
        Samples are index handles into the arena (no per-offspring copies) with env_params unpacked on demand.

        Multi-GPU (torch.distributed initialised, one process per GPU): this rank runs its contiguous
        block of tasks (shard.task_block).  Elites whose snapshot lives on another rank are moved first
        (place); at the end of the generation only the fp64 records (objectives + running statistics) are
        all-gathered, and each offspring's parameters / Adam state stay on the rank that produced them
        (remote handles elsewhere) until a later generation or the final writer needs them."""
        a = self.args
        P = len(task_batch)
        rank, ws = world()
        lo, hi = task_block(P, rank, ws)
        Pl = hi - lo
        if ws > 1:
            self.place([t.sample for t in task_batch], [owner_of(p, P, ws) for p in range(P)])
        total = int(a.num_env_steps) // a.num_steps // a.num_processes
        its = list(range(iteration, min(iteration + num_updates, total)))
        I = len(its)
        start_time = time.time() if start_time is None else start_time
        layout = self.layout
        L = layout.total
        tb = None
        if Pl > 0:
            tb = self._batch(Pl)
            self.load_tasks(tb, [t.sample for t in task_batch[lo:hi]],
                            [t.scalarization.weights.numpy() for t in task_batch[lo:hi]])
            step0 = [t.sample.snapshot.adam_step for t in task_batch[lo:hi]]
            tb.env_reset()  # envs are re-created and reset every generation (mopg.py:67-82)
            arena = torch.empty(I, 3, Pl, L, dtype=torch.float32, device=self.device)
            store = RowStore(arena, 'arena')
            rec = torch.empty(I, tb._stats64.numel(), dtype=torch.float64, device=self.device)
            objs_ar = torch.empty(I, Pl, tb.K, dtype=torch.float64, device=self.device)  # written by the evals
            for i, j in enumerate(its):
                lr = linear_lr(j, total, a.lr, a.lr_decay_ratio) if a.use_linear_lr_decay else a.lr
                noise = perms = None
                if self.rng == 'host':
                    noise, perms = host_draws(j, a.num_steps, a.num_processes, tb.A, a.ppo_epoch)
                tb.iteration(j, lr, noise=noise, perms=perms, carry=i > 0, overlap_eval=True, objs_out=objs_ar[i])
                arena[i].copy_(tb.state)
                tb.stats64_record(rec[i])
                if rank == 0 and a.rl_log_interval > 0 and (j + 1) % a.rl_log_interval == 0:
                    steps = (j + 1) * a.num_processes * a.num_steps
                    dt = time.time() - start_time
                    log(f'[RL] Updates {j + 1}, num timesteps {steps}, FPS {int(steps / max(dt, 1e-9))}, '
                        f'time {dt:.2f} seconds (x{P} tasks on {ws} device(s))')
            tb.wait_eval()
            if os.environ.get('PGM_DEBUG_TASKS'):
                print(f'[debug] generation at iteration {iteration}: P={P} local={Pl} iters={I} '
                      f'failed={int(tb.update_failed.item())}', flush=True)
        mismatch = None
        B = a.num_steps * a.num_processes
        per_iter = a.ppo_epoch * (B // (B // a.num_mini_batch))  # Adam steps of one iteration
        if tb is not None:
            got = tb.adam_step.cpu().numpy()
            want = np.asarray(step0) + I * per_iter
            if not np.array_equal(got, want):
                mismatch = f'rank {rank}: Adam step counts {got} != expected {want}'
        # a timed-out exchange or a lost Adam step never becomes an offspring (raised on every rank together)
        self.check_generation(tb, mismatch)
        probe = tb if tb is not None else None
        O, K = (probe.O, probe.K) if probe is not None else (layout.O, layout.K)
        if tb is not None:
            host_rec = rec.cpu().numpy()
            host_objs = objs_ar.cpu().numpy()
            stv = [tb.stat_views(host_rec[i], Pl) for i in range(I)]
        if ws > 1:  # generation boundary: objective + statistics records only (a few KB)
            width = K + 2 * O + 3 + 2 * K + 1
            mine = np.zeros((Pl, I, width))
            for i in range(I if Pl else 0):
                st = stv[i]
                mine[:, i] = np.concatenate([host_objs[i], st['ob_mean'], st['ob_var'], st['ob_count'][:, None],
                                             st['ret_mean'][:, None], st['ret_var'][:, None], st['ret_count'][:, None],
                                             st['obj_mean'], st['obj_var'], st['obj_count'][:, None]], 1)
            allr = allgather_rows(torch.from_numpy(mine).to(self.device), P).cpu().numpy()
            steps_all = allgather_rows(torch.tensor(step0 if Pl else [], dtype=torch.float64,
                                                    device=self.device).reshape(Pl), P).cpu().numpy()
        offspring = [[] for _ in range(P)]
        for p in range(P):
            own = owner_of(p, P, ws)
            q = p - lo
            for i in range(I):
                if ws == 1 or own == rank:
                    step = step0[q] + (i + 1) * per_iter
                    snap = DeviceSnapshot.in_arena(layout, store, i, q, step, owner=rank if ws > 1 else None)
                    objs = host_objs[i, q].copy()
                    fn = (lambda st=stv[i], q=q: self._env_params(st, q, O, K))
                else:
                    step = int(steps_all[p]) + (i + 1) * per_iter
                    snap = DeviceSnapshot.remote(layout, step, own)
                    r = allr[p, i]
                    objs = r[:K].copy()
                    st = self._split_record(r, O, K)
                    fn = (lambda st=st: self._env_params(st, 0, O, K))
                offspring[p].append(Sample.lazy(snap, fn, objs))
        return offspring

    @staticmethod
    def _split_record(r, O, K):
        """One all-gathered record row (objs, ob_mean/var, ob_count, ret mean/var/count, obj mean/var/count) ->
        the stat_views shape with one slot."""
        o = K
        out = {}
        for name, w in (('ob_mean', O), ('ob_var', O), ('ob_count', 1), ('ret_mean', 1), ('ret_var', 1),
                        ('ret_count', 1), ('obj_mean', K), ('obj_var', K), ('obj_count', 1)):
            v = r[o:o + w]
            out[name] = v[None] if w > 1 or name.startswith(('ob_m', 'ob_v', 'obj_m', 'obj_v')) else v
            o += w
        return out

    def evaluate_samples(self, samples, weights_batch):
        """Objectives of fresh samples (warm-up evaluation, morl/warm_up.py:69)."""
        tb = self._batch(len(samples))
        self.load_tasks(tb, samples, weights_batch)
        return tb.evaluate().cpu().numpy().copy()
