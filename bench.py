#!/usr/bin/env python3
"""Benchmark of the MOPG hot path on MI355X (BASELINE.json metric, SynthMO-Walker2d pop=40 per GPU).

One *step* = one MOPG iteration for every task on the GPU (morl/mopg.py:95-155): a T x N rollout
with the fused act + env + VecNormalize kernel, GAE, advantage scalarisation, ppo_epoch x
num_mini_batch Adam steps, the deterministic evaluation episode, and the generation-boundary
objective merge (RCCL all-gather of the per-task objective vectors when N > 1).
Counted env-steps = tasks x num_processes x num_steps per step (eval steps are not counted,
like the reference's FPS print, morl/mopg.py:159).

    python bench.py [--gpus N --steps K --warmup W]       # N > 1: starts the N ranks itself
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

At N > 1 the headline line is weak scaling (--tasks per GPU) and carries a second timed leg, `strong`: the
fixed population --strong-tasks (40) split over the ranks in task blocks (40 -> 20 / 10 / 5 per GPU).
"""
import argparse
import glob
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'env steps/sec (whole node) + hypervolume@budget, MO-Walker2d-v2 pop=40'
PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 (vector == f32-input MFMA), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='ranks (GPUs); without a launcher (WORLD_SIZE unset) bench.py starts them itself; under '
                         'torch.distributed.run it must equal WORLD_SIZE (default: WORLD_SIZE, else 1)')
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--env-name', default='MO-Walker2d-v2')
    ap.add_argument('--tasks', type=int, default=40,
                    help='tasks (policies) per GPU (--scaling weak) or in total (--scaling strong)')
    ap.add_argument('--scaling', choices=['weak', 'strong'], default='weak',
                    help='weak: --tasks on every GPU; strong: --tasks in total, split in contiguous blocks '
                         '(shard.task_block, the SURVEY §8(e) 40 -> 20/10/5 partition)')
    ap.add_argument('--num-processes', type=int, default=4)
    ap.add_argument('--num-steps', type=int, default=2048)
    ap.add_argument('--ppo-epoch', type=int, default=10)
    ap.add_argument('--num-mini-batch', type=int, default=32)
    ap.add_argument('--cpu-iters', type=int, default=16,
                    help='oracle iterations per process for cpu_baseline (16: ~20 s of wall time on the box)')
    ap.add_argument('--cpu-procs', type=int, default=15,
                    help='concurrent oracle processes: the 16-core host share of one GPU on the box minus the '
                         'bench process itself (the box allows 16 processes with the GPU open)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-overlap-eval', action='store_true', help='evaluate on the main stream (A/B)')
    ap.add_argument('--whole-run', dest='whole_run', action='store_true', default=None,
                    help='also time the whole PG-MORL run (pgmorl_amd.morl.run: warm-up, generations, selection, '
                         'writer) on Walker pop=40 with the reference budget (default: on at N=1)')
    ap.add_argument('--no-whole-run', dest='whole_run', action='store_false')
    ap.add_argument('--whole-run-steps', type=float, default=5e6,
                    help='--num-env-steps of the whole run (per task; scripts/walker2d-v2.py:38 uses 5e6)')
    ap.add_argument('--traffic-file', default=None,
                    help='PMC summary (scripts/pmc_summary.py) to quote as roofline.traffic; default: the newest '
                         'profiles/r0*_pmc_*.json whose workload matches this run')
    ap.add_argument('--strong-tasks', type=int, default=40,
                    help='global population of the strong-scaling leg (split over the ranks in task blocks)')
    ap.add_argument('--no-strong', action='store_true', help='skip the strong-scaling leg at N > 1')
    ap.add_argument('--stub-cpu', action='store_true', help=argparse.SUPPRESS)  # launcher tests (gloo, no GPU)
    return ap.parse_args()


def mflops_per_row(O, A, K, H=64):
    """M_f = 2(O*H + H^2) + H*A + H*K multiply-adds per row forward."""
    return 2 * (O * H + H * H) + H * A + H * K


def bytes_per_env_step(O, A, K, E):
    """Algorithmic HBM bytes per train env-step, fp32: rollout write, GAE read/write,
    advantage pass, E epoch re-reads of obs/action/old logp/old V/R/adv."""
    return 4 * ((O + A + 2 * K + 3) + (3 * K + 2) + (2 * K + 3) + E * (O + A + 2 * K + 2))


def _cpu_task(args, spec, task, barrier, q, cpu=None):
    """One reference-style task process (morl/morl.py:84-88): 1 thread (morl/morl.py:34), fp64 oracle, pinned to
    logical CPU ``cpu`` (one per physical core, _pick_cores) when given."""
    if cpu is not None:
        os.sched_setaffinity(0, {cpu})
    torch.set_num_threads(1)
    from oracle.mopg import initial_sample, mopg_worker
    from pgmorl_amd import envspec
    ns = argparse.Namespace(env_name=args.env_name, obj_num=spec['obj_num'], num_env_steps=10 ** 9, seed=0,
                            num_steps=args.num_steps, num_processes=args.num_processes, ppo_epoch=args.ppo_epoch,
                            num_mini_batch=args.num_mini_batch, clip_param=0.2, value_loss_coef=0.5,
                            entropy_coef=0.0, lr=3e-4, max_grad_norm=0.5, gamma=0.995, gae_lambda=0.95,
                            use_gae=True, use_proper_time_limits=True, ob_rms=True, obj_rms=True, raw=True,
                            eval_num=1, use_linear_lr_decay=True, lr_decay_ratio=1.0, layernorm=False)
    torch.manual_seed(task)
    sample = initial_sample(ns, spec)
    s0 = envspec.reset_table(spec['obs_dim'], 0, args.num_processes)
    s0e = envspec.reset_table(spec['obs_dim'], 0, 1)
    w = np.array([0.5] * spec['obj_num'])
    barrier.wait()
    t0 = time.time()
    mopg_worker(ns, spec, s0, s0e, sample, w, 0, args.cpu_iters)
    q.put((task, t0, time.time(), args.cpu_iters * args.num_processes * args.num_steps))


def _lscpu():
    try:
        import subprocess
        out = subprocess.run(['lscpu'], capture_output=True, text=True, timeout=10).stdout
        keep = ('Model name', 'Socket(s)', 'Core(s) per socket', 'Thread(s) per core', 'CPU(s)')
        return '; '.join(l.strip() for l in out.splitlines() if l.split(':')[0].strip() in keep)
    except Exception as e:  # lscpu absent: say so
        return f'lscpu unavailable ({e!r})'


def _cpu_busy(cpus, window=1.0):
    """Busy fraction of each logical CPU over ``window`` seconds (/proc/stat), {} if unreadable."""
    def snap():
        out = {}
        with open('/proc/stat') as f:
            for line in f:
                if line.startswith('cpu') and line[3].isdigit():
                    v = line.split()
                    c, t = int(v[0][3:]), [int(x) for x in v[1:]]
                    out[c] = (sum(t), t[3] + (t[4] if len(t) > 4 else 0))
        return out
    try:
        a = snap()
        time.sleep(window)
        b = snap()
    except OSError:
        return {}
    return {c: 1.0 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]) for c in cpus if c in a and c in b}


def _pick_cores(n):
    """n logical CPUs of the affinity mask on n distinct PHYSICAL cores (no SMT siblings: the topology from
    /sys/devices/system/cpu/cpu*/topology), the idlest cores first (busy fraction of both siblings over 1 s), so the
    baseline's processes neither share a core with each other nor land on a neighbour's busy core.  Returns
    (cpus, info); cpus None when the topology is unreadable."""
    avail = sorted(os.sched_getaffinity(0))
    cores = {}
    try:
        for c in avail:
            t = f'/sys/devices/system/cpu/cpu{c}/topology/'
            key = (int(open(t + 'physical_package_id').read()), int(open(t + 'core_id').read()))
            cores.setdefault(key, []).append(c)
    except (OSError, ValueError) as e:
        return None, {'pinning': f'none (topology unreadable: {e!r})'}
    busy = _cpu_busy(avail)
    own = os.sched_getaffinity(0)
    ranked = sorted(cores.items(), key=lambda kv: (max(busy.get(c, 0.0) for c in kv[1]), kv[0]))
    if len(ranked) < n:
        return None, {'pinning': f'none ({len(ranked)} physical cores < {n} processes)'}
    pick = [sibs[0] for _, sibs in ranked[:n]]
    return pick, {'pinning': 'one process per physical core, no SMT siblings, idlest cores first',
                  'cpus': pick, 'physical_cores_available': len(cores), 'own_mask_size': len(own),
                  'picked_busy_max': max(busy.get(c, 0.0) for _, sibs in ranked[:n] for c in sibs) if busy else None,
                  'all_cpus_busy_mean': float(np.mean(list(busy.values()))) if busy else None}


def cpu_baseline(args, spec, tasks):
    """The reference's CPU path, whole-node: one single-thread fp64 oracle process per task
    (morl/morl.py:34,84-88), as many concurrent processes as this GPU's host-core share (16 on the box,
    capped by the affinity mask and the population), each timing cpu_iters MOPG iterations of its task;
    value = all processes' train env-steps / the concurrent wall time.  The 96-vCPU figure scales the
    per-core rate to the reference's 96 Skylake vCPUs (README.md:92-94) -- an extrapolation, stated."""
    import multiprocessing as mp
    ncpu = len(os.sched_getaffinity(0))
    procs = max(1, min(args.cpu_procs, 15, ncpu, tasks))
    cpus, pin = _pick_cores(procs)
    load0 = os.getloadavg()
    ctx = mp.get_context('spawn')
    barrier, q = ctx.Barrier(procs), ctx.Queue()
    ps = [ctx.Process(target=_cpu_task, args=(args, spec, i, barrier, q, cpus[i] if cpus else None))
          for i in range(procs)]
    hide = {k: os.environ.get(k) for k in ('HIP_VISIBLE_DEVICES', 'ROCR_VISIBLE_DEVICES')}
    os.environ['HIP_VISIBLE_DEVICES'] = os.environ['ROCR_VISIBLE_DEVICES'] = ''  # CPU-only children
    try:
        for p in ps:
            p.start()
    finally:
        for k, v in hide.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = []
    while len(res) < procs:  # a dead worker ends the baseline instead of hanging the bench
        try:
            res.append(q.get(timeout=5))
        except Exception:
            if any(p.exitcode not in (None, 0) for p in ps):
                raise RuntimeError(f'cpu_baseline worker died: {[p.exitcode for p in ps]}')
    for p in ps:
        p.join(60)
    load1 = os.getloadavg()
    t0, t1 = min(r[1] for r in res), max(r[2] for r in res)
    steps = sum(r[3] for r in res)
    value = steps / (t1 - t0)
    rates = np.array([r[3] / (r[2] - r[1]) for r in res])  # each process's own rate (the spread across cores)
    # the per-core rate behind the 96-vCPU extrapolation: the MEDIAN process's own rate.  `value` (all steps / the
    # concurrent wall time) is set by the slowest process, and on the shared box (load average 25-31 from other
    # tenants, r06t) one process whose physical core another tenant starts using mid-run drags it 25 % down
    per_core = float(np.median(rates))
    return {'value': value, 'unit': 'env steps/sec', 'cores': procs, 'kind': 'port',
            'per_core': per_core, 'per_core_basis': 'median per-process rate', 'value_per_core': value / procs,
            'extrapolated_96vcpu': per_core * 96,
            'per_process': {'min': float(rates.min()), 'median': float(np.median(rates)), 'max': float(rates.max()),
                            'rel_sd': float(rates.std(ddof=1) / rates.mean()) if len(rates) > 1 else 0.0},
            'extrapolation': f'median per-process rate x 96 vCPUs (reference hardware, README.md:92-94)',
            'host': {'affinity_cpus': ncpu, 'os_cpu_count': os.cpu_count(), 'lscpu': _lscpu(),
                     'loadavg_before': list(load0), 'loadavg_after': list(load1)},
            'pinning': pin,
            'sample': f'{procs} concurrent single-thread processes x {args.cpu_iters} MOPG iterations each '
                      f'({steps} train env-steps, T={args.num_steps}, N={args.num_processes}, E={args.ppo_epoch}, '
                      f'M={args.num_mini_batch}, + eval) of the fp64 torch/numpy oracle, {t1 - t0:.1f} s wall'}


def hv_comparison(env_name):
    """The newest committed full-algorithm device-vs-oracle HV comparison at an equal budget for this env
    (scripts/hv_full.py: warm-up + prediction-guided generations on both sides, per seed), summarised."""
    key = {'MO-Walker2d-v2': 'walker', 'MO-Hopper-v2': 'hopper', 'MO-Hopper-v3': 'hopper3',
           'MO-Humanoid-v2': 'humanoid', 'MO-HalfCheetah-v2': 'cheetah'}.get(env_name)
    if key is None:
        return None
    import re

    def version(path):  # r<round>_hvfull<n>_<env>.json: newest round, then highest n (none = 1)
        m = re.match(r'r(\d+)_hvfull(\d*)_', os.path.basename(path))
        return (int(m.group(1)), int(m.group(2) or 1)) if m else (-1, -1)
    for dev in sorted(glob.glob(os.path.join(ROOT, 'profiles', f'r*_hvfull*_{key}.json')), key=version, reverse=True):
        orc = dev.replace(f'_{key}.json', f'_oracle_{key}.json').replace('oracle_oracle', 'oracle')
        if 'oracle' in os.path.basename(dev) or not os.path.exists(orc):
            continue
        d, o = json.load(open(dev)), json.load(open(orc))
        ho = {r['seed']: r['hv'] for r in o['runs']}
        pairs = [(r['hv'], ho[r['seed']]) for r in d['runs'] if r['seed'] in ho]
        if not pairs:
            continue
        hd_, ho_ = np.array(pairs).T
        # per-seed relative difference; when an oracle seed ends with an empty archive (HV 0: no point with every
        # objective >= 0 at this budget, Humanoid), every difference is taken relative to the oracle's mean HV, and
        # the verdict key changes with it (within_1pct_of_mean_at_95: not the per-seed statement); all oracle seeds
        # empty: no relative difference at all
        per_seed = bool((ho_ > 0).all())
        if not per_seed and ho_.mean() <= 0:
            rel, half = None, None
        else:
            scale = ho_ if per_seed else np.full_like(ho_, ho_.mean())
            rel = (hd_ - ho_) / scale
            half = None
            if len(rel) > 1:  # Student-t 95% interval of the mean per-seed difference
                from scipy import stats
                half = float(stats.t.ppf(0.975, len(rel) - 1) * rel.std(ddof=1) / np.sqrt(len(rel)))
        within = None if rel is None or half is None else bool(abs(rel.mean()) + half < 0.01)
        rec = d.get('device_sources_hash')
        return {'source': [os.path.relpath(dev, ROOT), os.path.relpath(orc, ROOT)], 'config': d.get('config'),
                'seeds': len(pairs), 'hv_rel_diff_per_seed': None if rel is None else [float(x) for x in rel],
                'hv_rel_diff_mean': None if rel is None else float(rel.mean()), 'ci95_half_width': half,
                'within_1pct_at_95': within if per_seed else None,
                'within_1pct_of_mean_at_95': None if per_seed else within,
                'hv_mean': {'device': float(hd_.mean()), 'oracle': float(ho_.mean())},
                'empty_archive_seeds': {'device': int((hd_ == 0).sum()), 'oracle': int((ho_ == 0).sum())},
                'normalised_by': 'per-seed oracle HV' if per_seed else 'mean oracle HV',
                # the device side's kernel sources (scripts/hv_full.py records them): null = not recorded (older run)
                'device_sources_hash': rec,
                'device_at_head': None if rec is None else rec == device_sources_hash()}
    return None


def hypervolume(args, history, budget):
    """HV of the EP over every offspring objective vector this run produced (morl/ep.py:23-31,
    morl/hypervolume.py), plus the committed device-vs-oracle comparison of the whole algorithm at an equal
    budget (hv_comparison), when one exists for this env."""
    from pgmorl_amd import pareto
    objs = torch.cat(history).cpu().numpy()
    idx = pareto.get_ep_indices(objs)
    hv = {'hv': pareto.compute_hypervolume(objs[idx]) if len(idx) else 0.0, 'ep_size': len(idx),
          'budget_env_steps': budget, 'rng': 'perf-mode device streams', 'ref_point': 0}
    cmp_ = hv_comparison(args.env_name)
    if cmp_ is not None:
        hv['vs_oracle_equal_budget'] = cmp_
    return hv


def whole_run(args, iter_value):
    """The whole-node metric of the reference (morl/morl.py:62-175 driven by morl/run.py): pgmorl_amd.morl.run
    end to end -- warm-up, every generation's MOPG on the device, EP / population / OptGraph, prediction-guided
    selection (native fits), the per-generation text dumps and the final EP policies -- on MO-Walker2d-v2 with
    pop = 40 (delta 1/39), update_iter 20, the reference's flags (scripts/walker2d-v2.py) and budget.  Timed
    from entering run() to its return (results tree complete); value = train env-steps / that wall time."""
    import tempfile
    from pgmorl_amd import pareto
    from pgmorl_amd.morl import run as morl_run
    from pgmorl_amd.run import get_parser, merge_argv
    save = tempfile.mkdtemp(prefix='pgm_whole_', dir=os.environ.get('TMPDIR', '/tmp'))
    argv = ['--env-name', 'MO-Walker2d-v2', '--obj-num', '2', '--num-env-steps', str(int(args.whole_run_steps)),
            '--warmup-iter', '80', '--update-iter', '20', '--min-weight', '0.0', '--max-weight', '1.0',
            '--delta-weight', repr(1.0 / 39), '--eval-num', '1', '--pbuffer-num', '100', '--pbuffer-size', '2',
            '--selection-method', 'prediction-guided', '--num-weight-candidates', '7', '--num-tasks', '40',
            '--sparsity', '1.0', '--obj-rms', '--ob-rms', '--raw', '--rl-log-interval', '0', '--seed', '0',
            '--save-dir', save]
    ns = get_parser().parse_args(merge_argv(argv))
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)  # morl/run.py:53
    import contextlib
    import io
    try:
        with contextlib.redirect_stdout(io.StringIO()):  # the selection's 'Too few candidates' notes
            t0 = time.perf_counter()
            ep = morl_run(ns, device="cuda", rng="device", log=None)
            wall = time.perf_counter() - t0
    finally:
        torch.set_default_dtype(old)
    tm = ep.timing
    objs = np.asarray(ep.obj_batch)
    import shutil
    shutil.rmtree(save, ignore_errors=True)
    v = tm['train_env_steps'] / wall
    per_gen = [(g['rl_s'], g['host_s']) for g in tm['generations']]
    gens = tm['generations']
    task_iters = sum(g['tasks'] * g['iters'] for g in gens)
    iters = sum(g['iters'] for g in gens)
    mean_tasks = task_iters / max(iters, 1)
    bench_iter_ms = 1e3 * args.tasks * args.num_processes * args.num_steps / iter_value
    g0 = gens[0] if gens else None  # the warm-up generation: all 40 tasks, like the iteration bench
    return {'value': v, 'unit': 'env steps/sec', 'wall_s': wall, 'final_s': tm.get('final_s'),
            # the selection's trajectory sets how many tasks a generation trains ('Too few candidates' shrinks it,
            # late generations can be empty), so the raw ratio to the 40-task bench mixes overhead with fewer tasks;
            # the overhead itself is the non-MOPG share of the wall time and the in-run iteration time at P = 40
            'tasks_per_generation': [g['tasks'] for g in gens], 'mean_active_tasks': mean_tasks,
            'overhead_share': (wall - tm['rl_s']) / wall,
            'warmup_iteration_ms': 1e3 * g0['rl_s'] / g0['iters'] if g0 and g0['iters'] else None,
            'bench_iteration_ms': bench_iter_ms,
            'vs_iteration_bench_per_task': (v / mean_tasks) / (iter_value / args.tasks) if mean_tasks else None,
            'generation_rl_host_s': per_gen, 'train_env_steps': tm['train_env_steps'],
            'generations': len(tm['generations']), 'mopg_s': tm['rl_s'], 'boundary_host_s': tm['host_s'],
            'init_s': tm['init_s'], 'host_share': tm['host_s'] / wall, 'vs_iteration_bench': v / iter_value,
            'hv': pareto.compute_hypervolume(objs) if len(objs) else 0.0, 'ep_size': int(len(objs)),
            'config': 'MO-Walker2d-v2 (SynthMO) pop=40, prediction-guided, warmup_iter 80, update_iter 20, '
                      f'num_env_steps {int(args.whole_run_steps)}, N=4, T=2048, E=10, M=32, device RNG, seed 0'}


# the sources each update-kernel family is compiled from (a PMC summary is only quoted for the exact sources it measured)
KERNEL_SOURCES = {
    'ppo_update_mfma_kernel': ['pgm_ppo_mfma.hip'], 'ppo_update_t16_kernel': ['pgm_ppo_mfma.hip'],
    'ppo_update_fs_kernel': ['pgm_ppo_fs.hip'], 'ppo_update_wide_kernel': ['pgm_ppo_wide.hip'],
}
KERNEL_HEADERS = ['pgm_common.hpp', 'pgm_mfma.hpp', 'pgm_ppo_shared.hpp', 'pgm_dispatch.hpp']


def device_sources_hash():
    """sha256 (16 hex digits) of every device-path source (csrc/ except the host-only pgm_host.cpp) and the C ABI
    header: what a device-side result (e.g. scripts/hv_full.py's HV runs) was produced with."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(ROOT, 'pgmorl_amd', 'csrc')
    for f in sorted(os.listdir(d)):
        if f.endswith(('.hip', '.hpp', '.cpp')) and f != 'pgm_host.cpp':
            with open(os.path.join(d, f), 'rb') as fp:
                h.update(f.encode() + b'\0' + fp.read())
    with open(os.path.join(ROOT, 'include', 'pgm_abi.h'), 'rb') as fp:
        h.update(fp.read())
    return h.hexdigest()[:16]


def kernel_source_hash(variant):
    """sha256 (16 hex digits) of the source files the update kernel named by ``variant`` (pgm_ppo_update_variant) is
    built from, plus the shared headers; None for an unknown family."""
    import hashlib
    fam = (variant or '').split(' ')[0]
    if fam not in KERNEL_SOURCES:
        return None
    h = hashlib.sha256()
    for f in KERNEL_SOURCES[fam] + KERNEL_HEADERS:
        with open(os.path.join(ROOT, 'pgmorl_amd', 'csrc', f), 'rb') as fp:
            h.update(f.encode() + b'\0' + fp.read())
    return h.hexdigest()[:16]


def pmc_traffic(args, workload, kernel):
    """roofline.traffic: HBM-side bytes per launch of the update kernel from the committed PMC summary of THIS
    workload (profiles/pmc_head.json: one entry per workload; A/B files are never listed there).  The entry must be
    for the same launch -- the full pgm_ppo_update_variant string (family, NS, R, two per CU) -- and for the same
    kernel sources (kernel_source_hash); otherwise (None, reason): a stale or other-variant PMC is never quoted."""
    if args.traffic_file:
        try:
            d = json.load(open(args.traffic_file))
        except Exception as e:
            return None, f'{args.traffic_file}: {e!r}'
        ent = {'variant': d.get('variant'), 'source_hash': d.get('source_hash'),
               'hbm_bytes_per_launch': d.get('hbm_bytes_per_launch'),
               'source': args.traffic_file} if d.get('workload') == workload else None
    else:
        try:
            ent = json.load(open(os.path.join(ROOT, 'profiles', 'pmc_head.json')))['entries'].get(workload)
        except Exception as e:
            return None, f'profiles/pmc_head.json: {e!r}'
    if not ent:
        return None, f'no PMC summary for {workload}'
    if not kernel or ent.get('variant') != kernel:
        return None, f"PMC summary {ent.get('source')} is for {ent.get('variant')!r}, not {kernel!r}"
    if ent.get('source_hash') != kernel_source_hash(kernel):
        return None, f"PMC summary {ent.get('source')} measured other kernel sources (stale)"
    return ent['hbm_bytes_per_launch'], ent['source']


def sq_evidence(workload, kernel):
    """The committed SQ-counter summary (scripts/sq_summary.py) of THIS workload's update launch from
    profiles/sq_head.json, under the same rule as pmc_traffic (same pgm_ppo_update_variant string, same kernel
    sources); (entry, None) or (None, reason)."""
    try:
        ent = json.load(open(os.path.join(ROOT, 'profiles', 'sq_head.json')))['entries'].get(workload)
    except Exception as e:
        return None, f'profiles/sq_head.json: {e!r}'
    if not ent:
        return None, f'no SQ summary for {workload}'
    if not kernel or ent.get('variant') != kernel:
        return None, f"SQ summary {ent.get('source')} is for {ent.get('variant')!r}, not {kernel!r}"
    if ent.get('source_hash') != kernel_source_hash(kernel):
        return None, f"SQ summary {ent.get('source')} measured other kernel sources (stale)"
    return ent, None


def limiter_of(sq):
    """What bounds the priced kernel by its own counters: the f32 MFMA pipe when it is busy at least half the wave
    lifetime, else latency (the dependent MFMA chains and the cross-CU hand-offs the waves wait on)."""
    if sq is None:
        return None
    busy = sq.get('mfma_busy_share')
    if busy is None:
        return None
    return 'mfma' if busy >= 0.5 else 'latency (hand-offs + dependent chains)'


def launch_ranks(n):
    """``python bench.py --gpus N`` with no launcher around it: start N rank processes of this script, one per GPU,
    with the environment torch.distributed.run would give them (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR =
    127.0.0.1 / MASTER_PORT), and return the first failing rank's exit code (0 when all succeed).  This parent never
    touches the GPU (no HIP call, no exec): each child selects its device before its first HIP call.  Only rank 0
    prints the JSON line; a rank that fails ends the others (SIGTERM, then SIGKILL after 30 s)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc, t_fail, live = 0, None, list(procs)
    while live:
        done = [(p, p.poll()) for p in live]
        done = [(p, c) for p, c in done if c is not None]
        for p, _ in done:
            live.remove(p)
        failed = [(procs.index(p), c) for p, c in done if c != 0]
        if failed and rc == 0:  # every rank found failed in the same sweep is named (a peer may exit in the same 0.1 s)
            rc, t_fail = (failed[0][1] if failed[0][1] > 0 else 1), time.time()
            for r, c in failed:
                print(f'bench.py: rank {r} exited with {c}; stopping the other ranks', file=sys.stderr)
            for q in live:
                q.terminate()
        if t_fail is not None and time.time() - t_fail > 30:
            for q in live:
                q.kill()
        time.sleep(0.1)
    return rc


def _gather_ints(x, dev):
    """All-gather one int per rank (list form: works on gloo and RCCL)."""
    t = torch.tensor([x], dtype=torch.int64, device=dev)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [int(p.item()) for p in parts]


def leg_gpu(args, spec, dev, rank, world, blocks, tag):
    """Time one population layout: rank r trains tasks blocks[r] = [lo, hi) of a population of blocks[-1][1].
    W warm-up iterations, then exactly K timed ones between a barrier + synchronize on both sides; returns
    {dt (max over ranks), upd_ms (max over ranks), history of gathered objective vectors, kernel}."""
    from pgmorl_amd.policy import new_policy
    from pgmorl_amd.runtime import TaskBatch
    from pgmorl_amd.shard import allreduce_max
    N, T, E, M = args.num_processes, args.num_steps, args.ppo_epoch, args.num_mini_batch
    G = blocks[-1][1]
    lo, hi = blocks[rank]
    P = hi - lo
    per = max(b - a for a, b in blocks)  # all-gather rows per rank (blocks padded to the largest)
    gathered = torch.zeros(world * per, spec['obj_num'], dtype=torch.float64, device=dev)
    mine = torch.zeros(per, spec['obj_num'], dtype=torch.float64, device=dev)
    tb = None
    if P > 0:
        tb = TaskBatch(args.env_name, P, num_processes=N, num_steps=T, ppo_epoch=E, num_mini_batch=M, device=dev)
        torch.manual_seed(rank * 1000)
        w = np.linspace(0, 1, G)[lo:hi]
        for p in range(P):
            pol = new_policy(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
            tb.set_task(p, pol.state_dict(), {}, None, [w[p], 1 - w[p]] if spec['obj_num'] == 2 else
                        np.ones(spec['obj_num']) / spec['obj_num'])
        tb.env_reset()
    total_updates = 5_000_000 // T // N
    history = []  # every iteration's gathered objective vectors (the offspring the EP is built from)
    overlap = not args.no_overlap_eval and tb is not None

    def step(j):
        # the evaluation of iteration j runs on the side stream beside iteration j+1's rollout; the objective
        # vectors are gathered on that stream behind it
        if tb is not None:
            tb.iteration(j, 3e-4 * (1 - j / total_updates), carry=True, overlap_eval=overlap)
        side = tb.eval_stream if overlap else torch.cuda.current_stream()
        with torch.cuda.stream(side):
            if world > 1:
                if tb is not None:
                    mine[:P].copy_(tb.objs)
                dist.all_gather_into_tensor(gathered, mine)
                history.append(torch.cat([gathered[r * per:r * per + b - a] for r, (a, b) in enumerate(blocks)]))
            else:
                gathered.copy_(tb.objs)
                history.append(gathered.clone())
            if overlap:
                # the next PPO update waits on this event: the RCCL gather never runs beside the update's
                # co-resident exchange workgroups
                tb._eval_done = torch.cuda.Event()
                tb._eval_done.record(side)

    j = 0
    for _ in range(args.warmup):
        step(j)
        j += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # per-launch duration of the dominant kernel (ppo_update) with events on the launch stream
    ev = []
    if tb is not None:
        orig_update = tb.ppo_update_launch

        def timed_update():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            orig_update()
            e.record()
            ev.append((s, e))

        tb.ppo_update_launch = timed_update
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(j)
        j += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if tb is not None:
        tb.ppo_update_launch = orig_update
        tb.check_update()  # a timed-out exchange invalidates the run: raises PGMError (after the timed region)
    upd_ms = float(np.mean([s.elapsed_time(e) for s, e in ev])) if ev else 0.0
    dt, upd_ms = allreduce_max([dt, upd_ms], dev)  # the slowest rank defines the step
    kernel = tb.update_variant() if tb is not None else None  # the launcher's own choice (pgm_ppo_update_variant)
    del tb
    torch.cuda.empty_cache()
    return {'dt': dt, 'upd_ms': upd_ms, 'P': P, 'history': history, 'kernel': kernel, 'tag': tag}


def leg_stub(args, spec, dev, rank, world, blocks, tag):
    """CPU stand-in for leg_gpu (--stub-cpu, tests only): the same rank plumbing, barriers, objective all-gather and
    max-over-ranks timing around a fixed sleep of 0.1 ms per task, so the launcher and the JSON assembly can be
    tested with gloo on a machine without a GPU.  Never a measurement."""
    from pgmorl_amd.shard import allreduce_max
    G = blocks[-1][1]
    lo, hi = blocks[rank]
    P = hi - lo
    per = max(b - a for a, b in blocks)
    history = []
    if os.environ.get('PGM_BENCH_STUB_FAIL_RANK') == str(rank):  # launcher test: one rank dies mid-run
        raise SystemExit(3)

    def step(j):
        time.sleep(1e-4 * P)
        mine = torch.zeros(per, spec['obj_num'], dtype=torch.float64)
        mine[:P] = torch.arange(lo, hi, dtype=torch.float64)[:, None] + j
        parts = [torch.empty_like(mine) for _ in range(world)] if world > 1 else [mine]
        if world > 1:
            dist.all_gather(parts, mine)
        history.append(torch.cat([parts[r][:b - a] for r, (a, b) in enumerate(blocks)]))

    for j in range(args.warmup):
        step(j)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for j in range(args.warmup, args.warmup + args.steps):
        step(j)
    if world > 1:
        dist.barrier()
    dt, upd_ms = allreduce_max([time.perf_counter() - t0, 0.0], dev)
    assert all(h.shape[0] == G for h in history)
    assert all(torch.equal(h[:, 0], torch.arange(G, dtype=torch.float64) + i) for i, h in enumerate(history))
    return {'dt': dt, 'upd_ms': upd_ms, 'P': P, 'history': history, 'kernel': 'stub', 'tag': tag}


def main():
    args = parse()
    env_ws = os.environ.get('WORLD_SIZE')
    if env_ws is None:
        if (args.gpus or 1) > 1:
            sys.exit(launch_ranks(args.gpus))
        world, rank, local = 1, 0, 0
    else:
        world, rank, local = int(env_ws), int(os.environ.get('RANK', '0')), int(os.environ.get('LOCAL_RANK', '0'))
        if args.gpus is not None and args.gpus != world:
            sys.exit(f'bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks; run '
                     f'`python bench.py --gpus N` (it starts the N ranks itself) or torch.distributed.run with '
                     f'--nproc-per-node equal to --gpus')
    if args.stub_cpu:
        dev = torch.device('cpu')
        if world > 1:
            dist.init_process_group('gloo')
        leg = leg_stub
    else:
        if world > 1:
            torch.cuda.set_device(local)
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        dev = torch.device('cuda', local)
        torch.cuda.set_device(dev)
        leg = leg_gpu
    n_gpus = 1
    if world > 1:  # the rank count the collectives actually see
        seen = _gather_ints(rank, dev)
        if sorted(seen) != list(range(world)):
            raise SystemExit(f'bench.py: ranks seen {seen} != range({world})')
        n_gpus = len(seen)

    from pgmorl_amd import envspec
    from pgmorl_amd.shard import task_block
    spec = envspec.make_spec(args.env_name)
    N, T, E, M = args.num_processes, args.num_steps, args.ppo_epoch, args.num_mini_batch
    if args.scaling == 'strong':  # a global population of --tasks, rank r trains its contiguous block
        blocks = [task_block(args.tasks, r, world) for r in range(world)]
    else:  # --tasks on every rank
        blocks = [(r * args.tasks, (r + 1) * args.tasks) for r in range(world)]
    if blocks[rank][1] <= blocks[rank][0] and args.scaling == 'weak':
        raise SystemExit(f'rank {rank}: no tasks')
    G = blocks[-1][1]
    main_leg = leg(args, spec, dev, rank, world, blocks, args.scaling)
    P = main_leg['P']
    dt, upd_ms = main_leg['dt'], main_leg['upd_ms']
    env_steps = G * N * T * args.steps  # every rank's tasks (the max-over-ranks time covers them all)
    value = env_steps / dt
    # the fixed population split over the ranks (pop 40 -> 40 / 20 / 10 / 5 per GPU), measured in the
    # same run: the strong-scaling curve the north star targets (>= 6x at 1 -> 8), beside the weak headline
    strong = None
    if not args.no_strong and args.scaling == 'weak' and world > 1:
        sblocks = [task_block(args.strong_tasks, r, world) for r in range(world)]
        sl = main_leg if sblocks == blocks else leg(args, spec, dev, rank, world, sblocks, 'strong')
        strong = {'global_tasks': args.strong_tasks, 'tasks_per_rank': [b - a for a, b in sblocks],
                  'value': args.strong_tasks * N * T * args.steps / sl['dt'], 'unit': 'env steps/sec',
                  'ms_per_step': sl['dt'] / args.steps * 1e3, 'update_ms': sl['upd_ms'],
                  'update_kernel_rank0': sl['kernel'], 'scaling': 'strong',
                  'note': 'same workload as the headline line' if sl is main_leg else
                          'second timed leg of this run (same steps / warm-up), max over ranks'}
        del sl
    mf = mflops_per_row(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
    upd_flop = P * T * N * E * 6 * mf          # fwd (2 M_f) + bwd (4 M_f) per row per epoch, one launch
    achieved = upd_flop / (upd_ms * 1e-3) / 1e12 if upd_ms > 0 else 0.0
    kernel = main_leg['kernel']
    traffic, traffic_src = pmc_traffic(args, f'{args.env_name}/P{P}/N{N}/T{T}/E{E}/M{M}', kernel)
    sq, sq_why = sq_evidence(f'{args.env_name}/P{P}/N{N}/T{T}/E{E}/M{M}', kernel)
    alg_bytes = P * T * N * E * 4 * (spec['obs_dim'] + spec['act_dim'] + 2 * spec['obj_num'] + 2)
    out = {
        'metric': METRIC, 'value': value, 'unit': 'env steps/sec', 'n_gpus': n_gpus, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt / args.steps * 1e3, 'higher_is_better': True, 'scaling': args.scaling,
        'vs_baseline': None, 'dtype': 'fp32', 'data': f"synthetic (SynthMO-{args.env_name.split('-')[1]} env, reference-order random init)",
        'config': {'workload': f'{args.env_name} (SynthMO) pop={G} ({args.scaling} scaling, {P} tasks on rank 0), '
                               f'N={N}, T={T}, ppo_epoch={E}, num_mini_batch={M}, eval_num=1, perf-mode device RNG',
                   'env': args.env_name, 'tasks_per_gpu': P, 'global_tasks': G, 'num_processes': N,
                   'num_steps': T, 'ppo_epoch': E, 'num_mini_batch': M, 'parallelism': f'task-sharded x{n_gpus}'},
        'roofline': {'bound': 'mfma', 'kernel': kernel, 'achieved': achieved,
                     'peak': PEAK_FP32_TFLOPS, 'unit': 'TFLOP/s', 'frac': achieved / PEAK_FP32_TFLOPS,
                     'traffic': traffic, 'traffic_source': traffic_src,
                     'traffic_vs_algorithmic': traffic / alg_bytes if traffic else None,
                     'avg_launch_ms': upd_ms, 'flop_per_launch': upd_flop, 'algorithmic_bytes_per_launch': alg_bytes,
                     # 'bound' names the roofline priced against (the dense f32 MFMA peak); 'limiter' what the kernel's
                     # own SQ counters say holds it below that (profiles/sq_head.json, same variant and sources)
                     'limiter': limiter_of(sq),
                     'mfma_busy': sq.get('mfma_busy_share') if sq else None,
                     'wait_any_share': sq.get('wait_any_share') if sq else None,
                     'sq_source': sq.get('source') if sq else sq_why},
        # whole-iteration view: env-steps/s x algorithmic FLOP (or bytes) per env-step vs peak
        'path_roofline': {'flop_per_env_step': 2 * mf * (1 + 3 * E),
                          'compute_frac': value * 2 * mf * (1 + 3 * E) / (n_gpus * PEAK_FP32_TFLOPS * 1e12),
                          'bytes_per_env_step': bytes_per_env_step(spec['obs_dim'], spec['act_dim'],
                                                                   spec['obj_num'], E),
                          'hbm_frac': value * bytes_per_env_step(spec['obs_dim'], spec['act_dim'], spec['obj_num'],
                                                                 E) / (n_gpus * PEAK_HBM_GBS * 1e9)},
    }
    if strong is not None:
        out['strong'] = strong
    if args.stub_cpu:
        out['data'] = 'STUB (--stub-cpu: launcher / rank plumbing test, not a measurement)'
    else:
        out['hypervolume'] = hypervolume(args, main_leg['history'], G * N * T * len(main_leg['history']))
    del main_leg
    if args.whole_run is None:
        args.whole_run = world == 1 and args.env_name == 'MO-Walker2d-v2' and args.scaling == 'weak' \
            and not args.stub_cpu
    if args.whole_run:
        torch.cuda.empty_cache()
        out['whole_run'] = whole_run(args, value)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.stub_cpu:
        out['cpu_baseline'] = cb = cpu_baseline(args, spec, G)
        out['vs_96vcpu_extrapolated'] = value / cb['extrapolated_96vcpu']
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
