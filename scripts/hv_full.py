"""Hypervolume at an equal env-step budget for the WHOLE PG-MORL algorithm: warm-up plus evolutionary
generations with prediction-guided selection (morl/morl.py:62-175), device vs the fp64 CPU oracle.

Both sides run the same host loop (pgmorl_amd.morl.run: EP, OptGraph, performance-buffer population,
prediction-guided selection, text dumps) from the same fp32-rounded reference-order initial policies with
the reference's RNG draws (torch.manual_seed(j) -> T x normal([N, A]), E x randperm(T N), morl/mopg.py:96);
only the MOPG back end differs: MOPGPopulation on the GPU (rng='host') or OracleMOPG, which trains every
task with the fp64 oracle MOPG_worker restatement in a process pool (one process per task, like
morl/morl.py:84-88).  Side 'oracle32' is the noise floor: the same fp64 oracle with each offspring's
parameters and Adam moments rounded to fp32 at the generation boundary (the device's storage precision),
compared against the plain oracle with --ref like the device side.  Side 'oracle_f32' is the precision arm: the
oracle with its policy, PPO losses, backward and Adam in fp32 (PGM_ORACLE_NET_DTYPE=float32, oracle/mopg.py NET),
envs / statistics / returns fp64 as on the device.  Each side picks its own elites from its own offspring, so the comparison is on the
budget-level quantities (HV of the final EP vs the origin, EP size, train env-steps), as
scripts/plot/ep_batch_visualize_2d.py:23-45 reports them.

    python scripts/hv_full.py oracle --env MO-Hopper-v2 --seeds 0 1 2 3 4 --out profiles/r02_hvfull_oracle_hopper.json
    python scripts/hv_full.py device --ref profiles/r02_hvfull_oracle_hopper.json --out profiles/r02_hvfull_hopper.json

Measurement harness (test infrastructure: it runs the oracle), not product code.
"""
import argparse
import json
import os
import sys
import tempfile
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pgmorl_amd import envspec, pareto  # noqa: E402
from pgmorl_amd.layout import STATE_KEYS, ParamLayout  # noqa: E402
from pgmorl_amd.run import get_parser, merge_argv  # noqa: E402
from pgmorl_amd.sample import DeviceSnapshot, RunningMeanStd, Sample  # noqa: E402

CONFIGS = {  # pop and the reference's per-env flags (scripts/*.py), iterations scaled to fit the budget
    'MO-Hopper-v2': dict(delta='0.25', tasks=5, N=1, warmup=10, update=5, gens=3, extra=[]),
    'MO-Walker2d-v2': dict(delta=str(1.0 / 39.0), tasks=40, N=4, warmup=4, update=3, gens=3, extra=[]),
    # scripts/hopper-v3.py: 3 objectives, delta 0.25 (15 warm-up tasks), pbuffer-num 20, sparsity 1e6
    'MO-Hopper-v3': dict(delta='0.25', tasks=15, N=4, warmup=4, update=3, gens=3,
                         extra=['--pbuffer-num', '20', '--sparsity', '1000000.0']),
    # scripts/halfcheetah-v2.py:37-51: delta 0.2 (6 warm-up tasks), num-tasks 6, eval-num 1; iterations scaled like Walker's
    'MO-HalfCheetah-v2': dict(delta='0.2', tasks=6, N=4, warmup=4, update=3, gens=3, extra=[]),
    # config 4 reduced (scripts/humanoid-v2.py: N = 8, gamma 0.99, eval_num 6, warm-up 200 / update 40 iterations at
    # delta 0.2): 5 tasks (delta 0.25), warm-up 40 + 2 generations x 10 = 60 iterations, past the iteration (~34)
    # where the archive of non-negative points first fills (profiles/r04_humanoid_hv.json)
    'MO-Humanoid-v2': dict(delta='0.25', tasks=5, N=8, warmup=40, update=10, gens=2,
                           extra=['--gamma', '0.99', '--eval-num', '6']),
    # config 1 at 2.8x the comparison budget (12 + 2 x 12 iterations): does the device-vs-oracle difference grow?
    # (warm-up >= update_iter: offspring enter the population every update_iter iterations, morl/morl.py:101, so a
    # shorter warm-up leaves it empty and no generation is selected)
    'MO-Walker2d-v2-long': dict(env='MO-Walker2d-v2', delta=str(1.0 / 39.0), tasks=40, N=4, warmup=12, update=12,
                                gens=2, extra=[]),
}


def make_args(env, seed, save_dir):
    c = CONFIGS[env]
    env = c.get('env', env)  # (a config key may name a budget variant of an env)
    T = 2048
    iters = c['warmup'] + c['gens'] * c['update']
    spec = envspec.make_spec(env)
    argv = ['--env-name', env, '--obj-num', str(spec['obj_num']), '--seed', str(seed),
            '--num-env-steps', str(iters * T * c['N']), '--num-processes', str(c['N']), '--num-steps', str(T),
            '--warmup-iter', str(c['warmup']), '--update-iter', str(c['update']), '--delta-weight', c['delta'],
            '--num-tasks', str(c['tasks']), '--selection-method', 'prediction-guided', '--pbuffer-num', '100',
            '--pbuffer-size', '2', '--num-weight-candidates', '7', '--sparsity', '1.0', '--obj-rms', '--ob-rms',
            '--raw', '--rl-log-interval', '0', '--save-dir', save_dir, '--rng', 'host'] + c['extra']
    return get_parser().parse_args(merge_argv(argv))


def _draws(T, N, A, E):
    def fn(j):
        torch.manual_seed(j)
        noise = torch.stack([torch.normal(torch.zeros(N, A, dtype=torch.float64), torch.ones(N, A, dtype=torch.float64))
                             for _ in range(T)])
        return noise.float().double(), [torch.randperm(T * N) for _ in range(E)]
    return fn


def _oracle_job(job):
    """One task's MOPG iterations with the fp64 oracle (one process, 1 thread: morl/morl.py:34,84-88)."""
    torch.set_num_threads(1)
    from oracle.mopg import initial_sample, mopg_worker
    from oracle.vecenv import RunningMeanStd as ORms
    a, flat, m, v, step, envp, w, iteration, num_updates = job
    args = argparse.Namespace(**a)
    spec = envspec.make_spec(args.env_name)
    lay = ParamLayout(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
    s = initial_sample(args, spec)
    s.actor_critic.load_state_dict(lay.unflatten(flat))
    osd = s.agent.optimizer.state_dict()
    osd['state'] = lay.adam_to_optimizer_state(m, v, step)
    s.agent.optimizer.load_state_dict(osd)
    for k, val in envp.items():
        if val is not None:
            r = ORms(shape=np.shape(val[0]))
            r.mean, r.var, r.count = np.array(val[0], dtype=np.float64), np.array(val[1], dtype=np.float64), float(val[2])
            s.env_params[k] = r
    s0_train = envspec.reset_table(spec['obs_dim'], 0, args.num_processes)
    s0_eval = envspec.reset_table(spec['obs_dim'], 0, args.eval_num)
    fn = _draws(args.num_steps, args.num_processes, spec['act_dim'], args.ppo_epoch)
    offs = mopg_worker(args, spec, s0_train, s0_eval, s, np.asarray(w), iteration, num_updates, noise_fn=fn)
    out = []
    for o in offs:
        st = o.agent.optimizer.state_dict()['state']
        ms = {key: st[i]['exp_avg'] for i, (key, _, _) in enumerate(STATE_KEYS)} if st else None
        vs = {key: st[i]['exp_avg_sq'] for i, (key, _, _) in enumerate(STATE_KEYS)} if st else None
        stp = int(float(st[0]['step'])) if st else 0
        zero = np.zeros(lay.total)
        ep = {k: (None if r is None else (np.array(r.mean), np.array(r.var), float(r.count)))
              for k, r in o.env_params.items()}
        out.append((np.asarray(o.objs, dtype=np.float64), lay.flatten(o.actor_critic.state_dict(), np.float64),
                    lay.flatten(ms, np.float64) if ms else zero, lay.flatten(vs, np.float64) if vs else zero, stp, ep))
    return out


def _env_params(ep):
    out = {}
    for k, val in ep.items():
        if val is None:
            out[k] = None
            continue
        r = RunningMeanStd(shape=np.shape(val[0]))
        r.mean, r.var, r.count = val[0], val[1], val[2]
        out[k] = r
    return out


class OracleMOPG:
    """MOPGPopulation's interface over the fp64 oracle (CPU, one process per task)."""

    def __init__(self, args, procs, round32=False):
        self.args, self.procs, self.round32 = args, procs, round32
        self.device = torch.device('cpu')
        spec = envspec.make_spec(args.env_name)
        self.spec, self._layout = spec, ParamLayout(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
        self.moved_bytes = 0

    @property
    def layout(self):
        return self._layout

    def _batch(self, P):
        return types.SimpleNamespace(layout=self._layout)

    def materialize(self, samples, dst=0):
        return 0

    def evaluate_samples(self, samples, weights_batch):
        from oracle.mopg import evaluation
        from oracle.policy import make_policy
        from oracle.vecenv import RunningMeanStd as ORms
        s0_eval = envspec.reset_table(self.spec['obs_dim'], 0, self.args.eval_num)
        out = []
        for s in samples:
            pol = make_policy(self.spec['obs_dim'], self.spec['act_dim'], self.spec['obj_num'])
            pol.load_state_dict(self._layout.unflatten(s.snapshot.params))
            r = ORms(shape=(self.spec['obs_dim'],))
            src = s.env_params.get('ob_rms')
            if src is not None:
                r.mean, r.var, r.count = np.array(src.mean), np.array(src.var), float(src.count)
            out.append(evaluation(self.args, self.spec, s0_eval, pol, r))
        return np.array(out)

    def run(self, task_batch, iteration, num_updates, start_time=None, log=print):
        import multiprocessing as mp
        a = dict(vars(self.args))
        jobs = []
        for t in task_batch:
            sn = t.sample.snapshot
            ep = {k: (None if r is None else (np.array(r.mean), np.array(r.var), float(r.count)))
                  for k, r in (t.sample.env_params or {}).items()}
            jobs.append((a, sn.params.double().numpy(), sn.adam_m.double().numpy(), sn.adam_v.double().numpy(),
                         sn.adam_step, ep, t.scalarization.weights.numpy(), iteration, num_updates))
        t0 = time.time()
        with mp.get_context('fork').Pool(min(self.procs, max(1, len(jobs)))) as pool:
            res = pool.map(_oracle_job, jobs)
        print(f'oracle generation: {len(jobs)} tasks x {num_updates} iterations from {iteration}, '
              f'{time.time() - t0:.0f} s', file=sys.stderr, flush=True)
        offspring = []
        for task_res in res:
            offs = []
            for objs, flat, m, v, step, ep in task_res:
                if self.round32:  # the device's storage precision at the generation boundary (noise floor)
                    flat, m, v = (x.astype(np.float32).astype(np.float64) for x in (flat, m, v))
                snap = DeviceSnapshot(self._layout, torch.from_numpy(flat), torch.from_numpy(m), torch.from_numpy(v), step)
                offs.append(Sample.from_snapshot(snap, _env_params(ep), objs))
            offspring.append(offs)
        return offspring


def run_side(side, env, seed, procs):
    from pgmorl_amd.morl import run
    with tempfile.TemporaryDirectory() as d:
        args = make_args(env, seed, d)
        runtime = OracleMOPG(args, procs, round32=side == 'oracle32') if side != 'device' else None
        t0 = time.time()
        ep = run(args, device='cuda' if side == 'device' else 'cpu', rng='host', log=lambda *m: None, runtime=runtime)
        dt = time.time() - t0
    front = np.asarray(ep.obj_batch).reshape(-1, args.obj_num)
    return {'seed': seed, 'hv': pareto.compute_hypervolume(front), 'ep_size': int(len(front)),
            'sparsity': pareto.compute_sparsity(front), 'train_env_steps': int(ep.timing['train_env_steps']),
            'generations': len(ep.timing['generations']), 'wall_s': dt, 'front': front.tolist()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('side', choices=['oracle', 'oracle32', 'oracle_f32', 'device'])
    ap.add_argument('--env', default='MO-Hopper-v2', choices=sorted(CONFIGS))
    ap.add_argument('--seeds', type=int, nargs='+', default=[0])
    ap.add_argument('--procs', type=int, default=7)
    ap.add_argument('--ref', help='oracle JSON (device side)')
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    if a.side != 'device':
        torch.set_num_threads(1)  # the host loop's own torch work (the warm-up evaluation): the pool has the cores
    if a.side == 'oracle_f32':  # before anything imports oracle.mopg (the pool workers fork from this process)
        os.environ['PGM_ORACLE_NET_DTYPE'] = 'float32'
    if a.ref:
        ref = json.load(open(a.ref))
        env, seeds = ref['env'], [r['seed'] for r in ref['runs']]
    else:
        env, seeds = a.env, a.seeds
    runs = [run_side(a.side, env, s, a.procs) for s in seeds]
    out = {'side': a.side, 'env': env, 'config': CONFIGS[env], 'runs': runs}
    if a.side == 'device':  # the kernel sources these runs used (bench.hv_comparison flags a stale comparison)
        from bench import device_sources_hash
        out['device_sources_hash'] = device_sources_hash()
    if a.ref:
        cmp = []
        for r, o in zip(runs, ref['runs']):
            cmp.append({'seed': r['seed'], 'side': a.side, 'hv_device': r['hv'], 'hv_oracle': o['hv'],
                        'hv_rel_diff': (r['hv'] - o['hv']) / max(abs(o['hv']), 1e-12),
                        'ep_size_device': r['ep_size'], 'ep_size_oracle': o['ep_size'],
                        'env_steps_device': r['train_env_steps'], 'env_steps_oracle': o['train_env_steps'],
                        'wall_s_device': r['wall_s'], 'wall_s_oracle': o['wall_s']})
        d = np.array([c['hv_rel_diff'] for c in cmp])
        out['vs_oracle'] = {'per_seed': cmp, 'mean_hv_rel_diff': float(d.mean()),
                            'worst_hv_rel_diff': float(d[np.argmax(np.abs(d))])}
    with open(a.out, 'w') as f:
        json.dump(out, f)
    print(json.dumps({k: v for k, v in out.items() if k != 'runs'} | {'hv': [r['hv'] for r in runs]}))


if __name__ == '__main__':
    main()
