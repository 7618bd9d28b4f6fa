"""The PG-MORL generation loop on top of the MI355X MOPG runtime (drop-in for morl/morl.py:28-239).

Warm-up (reference-order policy init, evaluation), then per generation: compose Tasks, run MOPG for
every task on the GPU (``MOPGPopulation.run`` replaces the process fan-out of morl/morl.py:79-99),
OptGraph / EP bookkeeping (morl/morl.py:101-125), task selection, and the per-generation text dumps
and final artefacts with the reference's formats and paths (morl/morl.py:179-239).

Selection: every method of morl/morl.py:128-169 -- 'prediction-guided' and 'random' through the
performance-buffer population of ``pgmorl_amd.population`` (morl/population_2d.py / population_3d.py),
'moead' over the population, 'ra' and 'pfa' over the last offspring.
"""
import json
import os
import pickle
import time
from copy import deepcopy

import numpy as np
import torch

from . import envspec
from .mopg import MOPGPopulation
from .pareto import EP, OptGraph, weight_grid
from .policy import new_policy
from .population import make_population
from .sample import DeviceSnapshot, RunningMeanStd, Sample, Task, WeightedSumScalarization, compact_snapshots
from .shard import world


def _fmt(n):
    return '{:5f}' + (n - 1) * ',{:5f}'


def initialize_warm_up_batch(args, runtime):
    """morl/warm_up.py:24-77: one reference-initialised policy + fresh env_params per weight, evaluated."""
    spec = envspec.make_spec(args.env_name)
    weights_batch = weight_grid(args.obj_num, args.delta_weight, args.min_weight, args.max_weight)
    samples, scal = [], []
    layout = runtime._batch(len(weights_batch)).layout
    dev = runtime.device
    for w in weights_batch:
        pol = new_policy(spec['obs_dim'], spec['act_dim'], args.obj_num)
        flat = torch.from_numpy(layout.flatten(pol.state_dict())).to(dev)
        snap = DeviceSnapshot(layout, flat, torch.zeros_like(flat), torch.zeros_like(flat), 0)
        env_params = {'ob_rms': RunningMeanStd(shape=(spec['obs_dim'],)) if args.ob_rms else None,
                      'ret_rms': RunningMeanStd(shape=()),
                      'obj_rms': RunningMeanStd(shape=()) if args.obj_rms else None}
        samples.append(Sample.from_snapshot(snap, env_params, optgraph_id=-1))
        scal.append(WeightedSumScalarization(num_objs=args.obj_num, weights=w))
    objs = runtime.evaluate_samples(samples, weights_batch)
    for s, o in zip(samples, objs):
        s.objs = o
    return samples, scal


def run(args, device='cuda', rng='device', log=print, runtime=None):
    """The generation loop.  ``runtime`` (default: MOPGPopulation on ``device``) is the MOPG back end: any
    object with MOPGPopulation's run / evaluate_samples / materialize / _batch(P).layout / device.
    ``log=None`` silences the progress lines (and skips formatting them)."""
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    t_start = time.perf_counter()
    runtime = MOPGPopulation(args, device=device, rng=rng) if runtime is None else runtime
    template = WeightedSumScalarization(num_objs=args.obj_num, weights=np.ones(args.obj_num) / args.obj_num)
    total_num_updates = int(args.num_env_steps) // args.num_steps // args.num_processes
    start_time = time.time()
    ep, opt_graph = EP(), OptGraph()
    population = make_population(args)
    if args.selection_method not in ('prediction-guided', 'random', 'ra', 'pfa', 'moead'):
        raise NotImplementedError(f'selection method {args.selection_method!r}')
    elite_batch, scalarization_batch = initialize_warm_up_batch(args, runtime)
    for s, sc in zip(elite_batch, scalarization_batch):
        s.optgraph_id = opt_graph.insert(deepcopy(sc.weights), deepcopy(s.objs), -1)
    # whole-run accounting: MOPG (device iterations, incl. the end-of-generation sync and record gather)
    # vs the generation-boundary host work (EP / population / OptGraph, selection, text dumps)
    timing = {'init_s': time.perf_counter() - t_start, 'rl_s': 0.0, 'host_s': 0.0, 'train_env_steps': 0,
              'generations': []}
    rl_num_updates = args.warmup_iter
    episode = iteration = 0
    rank, ws = world()
    writer = rank == 0  # every rank holds the same host state; one writes the results tree
    gen_writer = GenerationWriter() if writer else None
    ep_files = EPFileCache(os.path.join(args.save_dir, 'final'), gen_writer) if writer else None
    while iteration < total_num_updates:
        if log is not None:
            log('\n------------------------------- Warm-up Stage -------------------------------' if episode == 0 else
                f'\n-------------------- Evolutionary Stage: Generation {episode:3} --------------------')
        episode += 1
        task_batch = [Task(e, s) for e, s in zip(elite_batch, scalarization_batch)]
        t0 = time.perf_counter()
        all_offspring_batch = runtime.run(task_batch, iteration, rl_num_updates, start_time, log=log or (lambda *m: None))
        t1 = time.perf_counter()
        n_its = len(all_offspring_batch[0]) if all_offspring_batch else 0
        all_sample_batch, offspring_batch = [], []
        last_offspring_batch = [None] * len(task_batch)
        for task_id, offsprings in enumerate(all_offspring_batch):
            prev = task_batch[task_id].sample.optgraph_id
            w = task_batch[task_id].scalarization.weights.numpy()
            for i, s in enumerate(offsprings):
                all_sample_batch.append(s)
                if (i + 1) % args.update_iter == 0:
                    prev = opt_graph.insert(w, deepcopy(s.objs), prev)
                    s.optgraph_id = prev
                    offspring_batch.append(s)
            last_offspring_batch[task_id] = offsprings[-1]
        ep.update(all_sample_batch)
        population.update(offspring_batch)
        predicted_offspring_objs = []
        # ---------------- task selection (morl/morl.py:128-169)
        weights_batch = weight_grid(args.obj_num, args.delta_weight, args.min_weight, args.max_weight)
        if args.selection_method == 'ra':
            elite_batch = last_offspring_batch
            scalarization_batch = []
            for w in weights_batch:
                sc = deepcopy(template)
                sc.update_weights(w)
                scalarization_batch.append(sc)
        elif args.selection_method == 'pfa':
            if args.obj_num > 2:
                raise NotImplementedError('pfa needs 2 objectives')
            elite_batch = last_offspring_batch
            scalarization_batch = []
            ratio = (iteration + rl_num_updates + args.update_iter - args.warmup_iter) / \
                (total_num_updates - args.warmup_iter)
            ratio = np.clip(ratio, 0.0, 1.0)
            for i in np.arange(args.min_weight, args.max_weight + 0.5 * args.delta_weight, args.delta_weight):
                wv = np.clip(i + ratio * args.delta_weight, args.min_weight, args.max_weight)
                sc = deepcopy(template)
                sc.update_weights(np.array([abs(wv), abs(1.0 - wv)]))
                scalarization_batch.append(sc)
        elif args.selection_method == 'prediction-guided':
            elite_batch, scalarization_batch, predicted_offspring_objs = population.prediction_guided_selection(
                args, iteration, ep, opt_graph, template)
        elif args.selection_method == 'random':
            elite_batch, scalarization_batch = population.random_selection(args, template)
        else:  # moead: best population member per grid weight (morl/morl.py:128-140)
            elite_batch, scalarization_batch = [], []
            pool = population.sample_batch
            for w in weights_batch:
                sc = deepcopy(template)
                sc.update_weights(w)
                scalarization_batch.append(sc)
                best, best_v = None, -np.inf
                for s in pool:
                    v = sc.evaluate(torch.tensor(s.objs))
                    if v > best_v:
                        best, best_v = s, v
                elite_batch.append(best)
        if log is not None:
            log('Selected Tasks:')
            for e, sc in zip(elite_batch, scalarization_batch):
                log(f'objs = {e.objs}, weight = {sc.weights}')
        iteration = min(iteration + rl_num_updates, total_num_updates)
        rl_num_updates = args.update_iter
        if writer:
            gen_writer.submit(generation_record(
                args.save_dir, iteration, args.obj_num, ep, population, opt_graph, elite_batch, scalarization_batch,
                all_offspring_batch, predicted_offspring_objs if args.selection_method == 'prediction-guided' else None))
        # device memory follows the survivors (EP, population, next elites), not every offspring of the run: drop
        # this generation's offspring lists and gather the live snapshots out of its arena
        n_tasks = len(task_batch)
        steps = n_tasks * n_its * args.num_steps * args.num_processes
        del all_offspring_batch, all_sample_batch, offspring_batch, last_offspring_batch, task_batch
        compact_snapshots()
        if writer:  # the EP members' final files, written ahead on the writer thread while the next generation trains
            ep_files.update(ep)
        t2 = time.perf_counter()
        timing['rl_s'] += t1 - t0
        timing['host_s'] += t2 - t1
        timing['train_env_steps'] += steps
        timing['generations'].append({'iteration': iteration, 'tasks': n_tasks, 'iters': n_its,
                                      'rl_s': round(t1 - t0, 4), 'host_s': round(t2 - t1, 4)})
    t_final = time.perf_counter()
    runtime.materialize(list(ep.sample_batch), dst=0)  # collective: EP snapshots onto the writing rank
    if writer:
        gen_writer.join()
        write_final(args, ep, ep_files)
        timing['final_s'] = time.perf_counter() - t_final
        timing['wall_s'] = time.perf_counter() - t_start
        timing['env_steps_per_s_whole_run'] = timing['train_env_steps'] / timing['wall_s']
        timing['env_steps_per_s_rl_only'] = timing['train_env_steps'] / max(timing['rl_s'], 1e-9)
        timing['host_share'] = timing['host_s'] / timing['wall_s']
        timing['world_size'] = ws
        with open(os.path.join(args.save_dir, 'timing.json'), 'w') as fp:
            json.dump(timing, fp, indent=1)
        if log is not None:
            log(f"[timing] wall {timing['wall_s']:.2f} s: MOPG {timing['rl_s']:.2f} s, generation-boundary host "
                f"{timing['host_s']:.2f} s ({100 * timing['host_share']:.1f}%), {timing['train_env_steps']} train env-steps"
                f" -> {timing['env_steps_per_s_whole_run']:.4g} env-steps/s whole run")
    ep.timing = timing
    if ws > 1:
        torch.distributed.barrier()  # the results tree is complete before any rank returns
    return ep


def generation_record(save_dir, iteration, obj_num, ep, population, opt_graph, elite_batch, scalarization_batch,
                      all_offspring_batch, predicted_offspring_objs=None):
    """The data write_generation dumps, detached from the live EP / population / OptGraph (which the next
    generation mutates): plain lists of the (never mutated) objective / weight arrays."""
    return dict(save_dir=save_dir, iteration=iteration, obj_num=obj_num, ep_objs=ep.obj_batch,
                pop_objs=[s.objs for s in population.sample_batch],
                pop_ids=[s.optgraph_id for s in population.sample_batch],
                og_weights=list(opt_graph.weights), og_objs=list(opt_graph.objs), og_prev=list(opt_graph.prev),
                elites=[e.objs for e in elite_batch], weights=[sc.weights for sc in scalarization_batch],
                predictions=predicted_offspring_objs,
                offsprings=[s.objs for offs in all_offspring_batch for s in offs])


class GenerationWriter:
    """Writes the per-generation text dumps on a background thread (nothing in the loop reads them back), so
    the next generation's MOPG launches are not queued behind the formatting; join() before the final files."""

    def __init__(self):
        import queue
        import threading
        self._q = queue.Queue()
        self._err = None
        self._t = threading.Thread(target=self._loop, name='pgm-writer', daemon=True)
        self._t.start()

    def _loop(self):
        while True:
            rec = self._q.get()
            if rec is None:
                return
            try:
                rec() if callable(rec) else write_generation_record(rec)
            except BaseException as e:  # surfaced by join()
                self._err = e

    def submit(self, rec):
        self._q.put(rec)

    def join(self):
        self._q.put(None)
        self._t.join()
        if self._err is not None:
            raise self._err


def write_generation(save_dir, iteration, obj_num, ep, population, opt_graph, elite_batch, scalarization_batch,
                     all_offspring_batch, predicted_offspring_objs=None):
    """The per-generation text dumps of morl/morl.py:182-221: ep/objs.txt, population/{objs,optgraph}.txt,
    elites/{elites,weights,predictions,offsprings}.txt under save_dir/<iteration>/ ('{:5f}' CSV rows;
    optgraph.txt = node count, 'w;objs;prev' rows, population count, the members' node ids).
    predictions.txt is written only for prediction-guided selection (predicted_offspring_objs not None)."""
    write_generation_record(generation_record(save_dir, iteration, obj_num, ep, population, opt_graph, elite_batch,
                                              scalarization_batch, all_offspring_batch, predicted_offspring_objs))


def write_generation_record(r):
    """write_generation from a generation_record."""
    fmt = _fmt(r['obj_num'])
    base = os.path.join(r['save_dir'], str(r['iteration']))

    def rows(path, vecs):
        with open(path, 'w') as fp:
            for v in vecs:
                fp.write((fmt + '\n').format(*v))

    os.makedirs(os.path.join(base, 'ep'), exist_ok=True)
    rows(os.path.join(base, 'ep', 'objs.txt'), r['ep_objs'])
    os.makedirs(os.path.join(base, 'population'), exist_ok=True)
    rows(os.path.join(base, 'population', 'objs.txt'), r['pop_objs'])
    with open(os.path.join(base, 'population', 'optgraph.txt'), 'w') as fp:
        fp.write('{}\n'.format(len(r['og_objs'])))
        for w, o, pv in zip(r['og_weights'], r['og_objs'], r['og_prev']):
            fp.write((fmt + ';' + fmt + ';{}\n').format(*w, *o, pv))
        fp.write('{}\n'.format(len(r['pop_ids'])))
        for i in r['pop_ids']:
            fp.write('{}\n'.format(i))
    os.makedirs(os.path.join(base, 'elites'), exist_ok=True)
    rows(os.path.join(base, 'elites', 'elites.txt'), r['elites'])
    rows(os.path.join(base, 'elites', 'weights.txt'), r['weights'])
    if r['predictions'] is not None:
        rows(os.path.join(base, 'elites', 'predictions.txt'), r['predictions'])
    rows(os.path.join(base, 'elites', 'offsprings.txt'), r['offsprings'])


class _StateDictWriter:
    """torch.save of many state_dicts with identical keys, shapes and dtypes (the EP policies), without re-pickling:
    the first is saved by torch.save into memory; every later file is that zip image with the tensor records' bytes
    replaced (torch.save stores them uncompressed, 64-B aligned, one record per storage in state_dict order) and each
    patched record's CRC-32 recomputed (zlib.crc32, local header and central directory), so every file is a valid zip
    exactly like torch.save's.  Before the writer is used, a templated image of a probe state_dict (same keys, shapes
    and dtypes, different values) is read back with torch.load(weights_only=True) and compared, synchronously; any
    mismatch makes ``ok`` False and every file goes through torch.save."""

    def __init__(self, sd):
        import io
        import zipfile
        self.keys = list(sd)
        b = io.BytesIO()
        self.crc = True
        torch.save(sd, b)
        self.tmpl = b.getvalue()
        self.ok = False
        try:
            z = zipfile.ZipFile(io.BytesIO(self.tmpl))
            info = {i.filename: i for i in z.infolist()}
            prefix = z.infolist()[0].filename.split('/')[0]
            cd = {}  # central-directory record offset of each member
            pos = self.tmpl.rfind(b'PK\x05\x06')
            cd_off = int.from_bytes(self.tmpl[pos + 16:pos + 20], 'little')
            n = int.from_bytes(self.tmpl[pos + 10:pos + 12], 'little')
            o = cd_off
            for _ in range(n):
                fl, el, cl = (int.from_bytes(self.tmpl[o + k:o + k + 2], 'little') for k in (28, 30, 32))
                cd[self.tmpl[o + 46:o + 46 + fl].decode()] = o
                o += 46 + fl + el + cl
            self.rec = []
            for k, key in enumerate(self.keys):
                zi = info[f'{prefix}/data/{k}']
                h = zi.header_offset
                fl, el = (int.from_bytes(self.tmpl[h + k2:h + k2 + 2], 'little') for k2 in (26, 28))
                t = sd[key]
                if zi.compress_type != 0 or zi.file_size != t.numel() * t.element_size():
                    return
                self.rec.append((h + 30 + fl + el, zi.file_size, h + 14, cd[zi.filename] + 16))
            self.ok = True
            self._self_check(sd)
        except Exception:
            self.ok = False

    def _self_check(self, sd):
        """The templated image of a probe state_dict must torch.load to exactly that state_dict."""
        import io
        probe = {}
        for i, key in enumerate(self.keys):
            t = sd[key].detach()
            probe[key] = (torch.arange(t.numel(), dtype=torch.float64).reshape(t.shape) * 0.5 + i + 1).to(t.dtype)
        got = torch.load(io.BytesIO(bytes(self._render([probe[k].numpy() for k in self.keys]))), weights_only=True)
        self.ok = list(got) == self.keys and all(torch.equal(got[k], probe[k]) and got[k].dtype == probe[k].dtype
                                                 for k in self.keys)

    def save(self, sd, path):
        if not self.ok:
            torch.save(sd, path)
            return
        self.save_records([sd[key].detach().contiguous().numpy() for key in self.keys], path)

    def save_records(self, arrays, path):
        """The templated file from the state_dict's tensors as numpy arrays (state_dict order, exact dtypes)."""
        buf = self._render(arrays)
        with open(path, 'wb') as fp:
            fp.write(buf)

    def _render(self, arrays):
        import zlib
        buf = bytearray(self.tmpl)
        for (off, size, lcrc, ccrc), arr in zip(self.rec, arrays):
            data = memoryview(np.ascontiguousarray(arr)).cast('B')
            if data.nbytes != size:  # a slice assignment of another length would resize the zip silently
                raise ValueError(f'EP template record of {size} bytes given {data.nbytes} bytes '
                                 f'({getattr(arr, "dtype", "?")} {getattr(arr, "shape", "?")})')
            buf[off:off + size] = data
            if self.crc:
                crc = zlib.crc32(data).to_bytes(4, 'little')
                buf[lcrc:lcrc + 4] = crc
                buf[ccrc:ccrc + 4] = crc
        return buf

    def verify(self, sd, path):
        """torch.load of a templated file must equal its state_dict bit for bit (else: torch.save from now on)."""
        if not self.ok:
            return
        got = torch.load(path, weights_only=True)
        if list(got) != self.keys or not all(torch.equal(got[k], sd[k]) and got[k].dtype == sd[k].dtype
                                             for k in self.keys):
            self.ok = False
            torch.save(sd, path)


class EPFileCache:
    """The final EP files (EP_policy_i.pt, EP_env_params_i.pkl, morl/morl.py:223-230) of every archive member,
    written AHEAD: at each generation boundary the members that entered the EP get their two files under
    final/.ep_cache/<uid>.{pt,pkl} on the background writer thread (one device->host copy of their parameters on the
    main thread), and the files of members that left are deleted there too.  write_final then only renames each
    final member's pair to its index (os.replace) instead of serialising thousands of policies at the end of the run.
    Snapshots are immutable, so a member's files never go stale.  Members whose snapshot lives on another rank
    (multi-GPU) are written by write_final after the final gather, as before."""

    def __init__(self, final_dir, gen_writer):
        import itertools
        self.dir = os.path.join(final_dir, '.ep_cache')
        self.writer = gen_writer
        self.files = {}  # uid -> (pt path, pkl path), written or queued
        self.next_uid = itertools.count()
        self.sdw = None

    def _paths(self, uid):
        return os.path.join(self.dir, f'{uid}.pt'), os.path.join(self.dir, f'{uid}.pkl')

    def update(self, ep):
        members = list(ep.sample_batch)
        live = set()
        new = []
        for smp in members:
            uid = getattr(smp, '_ep_uid', None)
            if uid is None:
                uid = smp._ep_uid = next(self.next_uid)
            live.add(uid)
            if uid not in self.files and smp.snapshot.is_local:
                new.append((uid, smp))
        gone = [self.files.pop(u) for u in [u for u in self.files if u not in live]]
        if new:
            layout = new[0][1].snapshot.layout
            # the new members' flat parameters in ONE device->host copy; the per-key fp64 / transposed blocks are
            # made from it on the writer thread (numpy, the same values as the device conversion)
            flats = torch.stack([smp.snapshot.params for _, smp in new]).cpu().numpy()
            if self.sdw is None:
                self.sdw = _StateDictWriter(layout.unflatten(flats[0]))
            sdw = self.sdw  # (its template was verified when it was built: the path chosen here is final)
            envs = [smp.env_params for _, smp in new]
            smps = [smp for _, smp in new]
            paths = [self._paths(uid) for uid, _ in new]
            for (uid, _), pp in zip(new, paths):
                self.files[uid] = pp

            def job():
                os.makedirs(self.dir, exist_ok=True)
                blocks = layout.unflatten_batch(flats) if sdw.ok else None
                sds = None if blocks is not None else [layout.unflatten(f) for f in flats]
                for i, (pt, pkl) in enumerate(paths):
                    if blocks is not None:
                        sdw.save_records([b[i] for b in blocks], pt)
                    else:
                        sdw.save(sds[i], pt)
                    with open(pkl, 'wb') as fp:
                        pickle.dump(envs[i], fp)
                    smps[i]._env_line = _env_params_line(envs[i])  # env_params.txt's line, ahead too
            self.writer.submit(job)
        if gone:
            def drop():
                for pt, pkl in gone:
                    for f in (pt, pkl):
                        try:
                            os.remove(f)
                        except FileNotFoundError:
                            pass
            self.writer.submit(drop)

    def take(self, smp, i, final):
        """Move a written member's pair to its final index; False when it has none (write it directly)."""
        uid = getattr(smp, '_ep_uid', None)
        pp = self.files.pop(uid, None) if uid is not None else None
        if pp is None or not os.path.exists(pp[0]) or not os.path.exists(pp[1]):
            return False
        os.replace(pp[0], os.path.join(final, f'EP_policy_{i}.pt'))
        os.replace(pp[1], os.path.join(final, f'EP_env_params_{i}.pkl'))
        return True

    def close(self):
        import shutil
        shutil.rmtree(self.dir, ignore_errors=True)
        self.files.clear()


def _env_params_line(env_params):
    """One line of final/env_params.txt (morl/morl.py:236-239): numpy's own str() of obj_rms mean / var."""
    r = env_params.get('obj_rms') if env_params else None
    return None if r is None else 'obj_rms: mean: {} var: {}\n'.format(r.mean, r.var)


def write_final(args, ep, cache=None):
    """morl/morl.py:223-245: final/EP_policy_i.pt, EP_env_params_i.pkl, objs.txt, env_params.txt.  With ``cache``
    (an EPFileCache whose writer thread has been joined) members written ahead are renamed into place."""
    fmt = _fmt(args.obj_num)
    final = os.path.join(args.save_dir, 'final')
    os.makedirs(final, exist_ok=True)
    samples = list(ep.sample_batch)
    if cache is not None:
        todo = [i for i, smp in enumerate(samples) if not cache.take(smp, i, final)]
        cache.close()
    else:
        todo = list(range(len(samples)))
    if todo:  # every remaining EP policy's flat parameters in ONE device->host copy, then the reference state_dicts
        snaps = [samples[i].snapshot for i in todo]
        flats_dev = torch.stack([sn.params for sn in snaps])
        flats = None
        envs = [samples[i].env_params for i in todo]
        layout = snaps[0].layout
        sd0 = layout.unflatten(flats_dev[0])
        sdw = _StateDictWriter(sd0)
        p0 = os.path.join(final, f'EP_policy_{todo[0]}.pt')
        sdw.save(sd0, p0)
        sdw.verify(sd0, p0)

        # every policy's tensors at once: per state_dict key, the [E, *shape] fp64 block (transposed back from the
        # device's [in][out] weights) -- the per-file work is then byte copies and CRCs
        blocks = layout.unflatten_batch(flats_dev) if sdw.ok else None
        if blocks is None:
            flats = flats_dev.cpu().numpy()

        def save(j):
            i = todo[j]
            if j:
                path = os.path.join(final, f'EP_policy_{i}.pt')
                if blocks is not None:
                    sdw.save_records([b[j] for b in blocks], path)
                else:
                    sdw.save(layout.unflatten(flats[j]), path)
            with open(os.path.join(final, f'EP_env_params_{i}.pkl'), 'wb') as fp:
                pickle.dump(envs[j], fp)
        # file creation and writes release the GIL: two writer threads overlap them with the Python work (one EP
        # can hold thousands of policies; more threads only contend for the GIL)
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=2) as ex:
            list(ex.map(save, range(len(todo))))
    with open(os.path.join(final, 'objs.txt'), 'w') as fp:
        for obj in ep.obj_batch:
            fp.write((fmt + '\n').format(*obj))
    if args.obj_rms:
        with open(os.path.join(final, 'env_params.txt'), 'w') as fp:
            for s in ep.sample_batch:
                line = getattr(s, '_env_line', None)  # (formatted on the writer thread by EPFileCache)
                fp.write(line if line is not None else _env_params_line(s.env_params))
