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
from .sample import DeviceSnapshot, RunningMeanStd, Sample
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
        a = self.args
        if self.tb is None or self.tb.P != P:
            self.tb = TaskBatch(a.env_name, P, num_processes=a.num_processes, num_steps=a.num_steps, seed=a.seed,
                                eval_num=a.eval_num, gamma=a.gamma, gae_lambda=a.gae_lambda, use_gae=a.use_gae,
                                use_proper_time_limits=a.use_proper_time_limits, ob_rms=a.ob_rms,
                                obj_rms=a.obj_rms, raw=a.raw, clip_param=a.clip_param, ppo_epoch=a.ppo_epoch,
                                num_mini_batch=a.num_mini_batch, value_loss_coef=a.value_loss_coef,
                                entropy_coef=a.entropy_coef, max_grad_norm=a.max_grad_norm, device=self.device)
        return self.tb

    def load_task(self, tb, p, sample, weights):
        snap = sample.snapshot
        tb.params[p].copy_(snap.params)
        tb.adam_m[p].copy_(snap.adam_m)
        tb.adam_v[p].copy_(snap.adam_v)
        tb.adam_step[p] = snap.adam_step
        tb.weights[p].copy_(torch.as_tensor(np.asarray(weights, dtype=np.float64)))
        ep = sample.env_params or {}
        tb.set_env_params(p, {k: v for k, v in ep.items() if v is not None})

    def _record_width(self, tb):
        return 3 * tb.K + 2 * tb.O + 6

    def _records(self, tb):
        """Per-task fp64 record of one iteration: objs[K], ob_mean/var[O], ob_count, ret mean/var/count,
        obj_mean/var[K], obj_count, adam_step (the snapshot fields of mopg.py:146-155)."""
        col = lambda x: x.reshape(tb.P, -1).to(torch.float64)
        return torch.cat([col(tb.objs), col(tb.ob_mean), col(tb.ob_var), col(tb.ob_count), col(tb.ret_mean),
                          col(tb.ret_var), col(tb.ret_count), col(tb.obj_mean), col(tb.obj_var), col(tb.obj_count),
                          col(tb.adam_step)], 1)

    def _unpack(self, rec, O, K):
        """One host record row -> (objs, env_params RunningMeanStd copies, adam_step)."""
        o = 0

        def take(n):
            nonlocal o
            v = rec[o:o + n].copy()
            o += n
            return v
        objs, ob_mean, ob_var, ob_count = take(K), take(O), take(O), take(1)[0]
        ret_mean, ret_var, ret_count = take(1)[0], take(1)[0], take(1)[0]
        obj_mean, obj_var, obj_count, step = take(K), take(K), take(1)[0], take(1)[0]
        ep = {'ob_rms': None, 'ret_rms': None, 'obj_rms': None}
        if self.args.ob_rms:
            r = RunningMeanStd(shape=(O,))
            r.mean, r.var, r.count = ob_mean, ob_var, float(ob_count)
            ep['ob_rms'] = r
        r = RunningMeanStd(shape=())
        r.mean, r.var, r.count = np.float64(ret_mean), np.float64(ret_var), float(ret_count)
        ep['ret_rms'] = r
        if self.args.obj_rms:
            r = RunningMeanStd(shape=())
            r.mean, r.var, r.count = obj_mean, obj_var, float(obj_count)
            ep['obj_rms'] = r
        return objs, ep, int(step)

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

    def run(self, task_batch, iteration, num_updates, start_time=None, log=print):
        """Every task's MOPG iterations [iteration, iteration + num_updates) -> all_offspring_batch.

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
        start_time = time.time() if start_time is None else start_time
        snaps32, recs = [], []
        tb = None
        if Pl > 0:
            tb = self._batch(Pl)
            tb.reset_stats()
            for p, task in enumerate(task_batch[lo:hi]):
                self.load_task(tb, p, task.sample, task.scalarization.weights.numpy())
            tb.env_reset()  # envs are re-created and reset every generation (mopg.py:67-82)
            objs_i = []  # each iteration's evaluation output (written on the overlapped eval stream)
            for i, j in enumerate(its):
                lr = linear_lr(j, total, a.lr, a.lr_decay_ratio) if a.use_linear_lr_decay else a.lr
                noise = perms = None
                if self.rng == 'host':
                    noise, perms = host_draws(j, a.num_steps, a.num_processes, tb.A, a.ppo_epoch)
                objs_i.append(torch.empty(Pl, tb.K, dtype=torch.float64, device=self.device))
                tb.iteration(j, lr, noise=noise, perms=perms, carry=i > 0, overlap_eval=True, objs_out=objs_i[-1])
                snaps32.append(torch.stack([tb.params, tb.adam_m, tb.adam_v], 1))  # [Pl, 3, L] (a copy)
                recs.append(self._records(tb))  # objs columns filled from objs_i below
                if rank == 0 and a.rl_log_interval > 0 and (j + 1) % a.rl_log_interval == 0:
                    steps = (j + 1) * a.num_processes * a.num_steps
                    dt = time.time() - start_time
                    log(f'[RL] Updates {j + 1}, num timesteps {steps}, FPS {int(steps / max(dt, 1e-9))}, '
                        f'time {dt:.2f} seconds (x{P} tasks on {ws} device(s))')
            tb.wait_eval()
            if os.environ.get('PGM_DEBUG_TASKS'):
                print(f'[debug] generation at iteration {iteration}: P={P} local={Pl} iters={len(its)} '
                      f'failed={int(tb.update_failed.item())}', flush=True)
            tb.check_update()  # a timed-out exchange never becomes an offspring (raises PGMError)
            for rec, ob in zip(recs, objs_i):
                rec[:, :tb.K] = ob
        probe = self._batch(1) if tb is None else tb
        L, O, K = probe.layout.total, probe.O, probe.K
        if recs:
            r64 = torch.stack(recs, 1)  # [Pl, I, S]
        else:
            r64 = torch.zeros(Pl, len(its), self._record_width(probe), dtype=torch.float64, device=self.device)
        if ws > 1:  # generation boundary: objective + statistics records only (a few KB)
            r64 = allgather_rows(r64, P)
        host = r64.cpu().numpy()
        offspring = [[] for _ in range(P)]
        for p in range(P):
            own = owner_of(p, P, ws)
            for i in range(len(its)):
                objs, envp, step = self._unpack(host[p, i], O, K)
                if own == rank:  # each survivor pins only its own [3, L] (the stacked block is freed)
                    blk = snaps32[i][p - lo].clone()  # [3, L]
                    snap = DeviceSnapshot(probe.layout, blk[0], blk[1], blk[2], step, owner=rank if ws > 1 else None)
                else:
                    snap = DeviceSnapshot.remote(probe.layout, step, own)
                offspring[p].append(Sample.from_snapshot(snap, envp, objs))
        return offspring

    def evaluate_samples(self, samples, weights_batch):
        """Objectives of fresh samples (warm-up evaluation, morl/warm_up.py:69)."""
        tb = self._batch(len(samples))
        tb.reset_stats()
        for p, (s, w) in enumerate(zip(samples, weights_batch)):
            self.load_task(tb, p, s, w)
        return tb.evaluate().cpu().numpy().copy()
