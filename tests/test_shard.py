"""Multi-rank path on CPU: task blocks and the generation-boundary all-gather over gloo, world_size 2 and 3
(the GPU run uses the same code over RCCL)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pgmorl_amd.shard import allgather_rows, allreduce_max, task_block


def test_task_blocks_cover_every_task_once():
    for P in (1, 5, 40, 160, 210):
        for G in (1, 2, 3, 4, 8):
            blocks = [task_block(P, r, G) for r in range(G)]
            owned = [p for lo, hi in blocks for p in range(lo, hi)]
            assert owned == list(range(P))
            assert max(hi - lo for lo, hi in blocks) == -(-P // G)
    assert [task_block(40, r, 8) for r in range(8)] == [(5 * r, 5 * r + 5) for r in range(8)]


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, ws, port, P, errq):
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        dist.init_process_group('gloo', rank=rank, world_size=ws)
        lo, hi = task_block(P, rank, ws)
        # per-task offspring payloads: [P_local, iters, 3, L] fp32 snapshots and [P_local, iters, S] fp64 records
        s32 = torch.stack([torch.full((4, 3, 7), float(p)) + torch.arange(7.0) for p in range(lo, hi)]) \
            if hi > lo else torch.zeros(0, 4, 3, 7)
        r64 = torch.stack([torch.arange(5, dtype=torch.float64) * 1e-3 + p for p in range(lo, hi)]) \
            if hi > lo else torch.zeros(0, 5, dtype=torch.float64)
        g32, g64 = allgather_rows(s32, P), allgather_rows(r64, P)
        assert g32.shape == (P, 4, 3, 7) and g64.shape == (P, 5)
        for p in range(P):
            assert torch.equal(g32[p], torch.full((4, 3, 7), float(p)) + torch.arange(7.0))
            assert torch.equal(g64[p], torch.arange(5, dtype=torch.float64) * 1e-3 + p)
        t = allreduce_max([rank + 0.5, -rank], 'cpu')
        assert t == [ws - 0.5, 0.0]
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surfaced by the parent
        errq.put(f'rank {rank}: {e!r}')
        raise


@pytest.mark.parametrize('ws,P', [(2, 40), (2, 5), (3, 7), (3, 2)])
def test_allgather_rows_gloo(ws, P):
    ctx = mp.get_context('spawn')
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, P, errq))
             for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _selection_worker(rank, ws, port, K, errq):
    """Generation boundary on ws ranks (morl/morl.py:100-169): every rank owns a block of the offspring,
    all-gathers the (objs, optgraph_id) rows, then runs prediction-guided selection itself from the same
    seed; every rank must pick the same elites, weights and predictions as the single-process run."""
    try:
        import numpy as np
        from pgmorl_amd import pareto, population
        from pgmorl_amd.sample import WeightedSumScalarization
        from tests.test_population import _EP, _S, _args, _history
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        dist.init_process_group('gloo', rank=rank, world_size=ws)
        og, offspring = _history(K, 1)
        P = len(offspring)
        lo, hi = task_block(P, rank, ws)
        mine = torch.tensor([list(s.objs) + [s.optgraph_id] for s in offspring[lo:hi]], dtype=torch.float64)
        rows = allgather_rows(mine.reshape(hi - lo, K + 1), P).numpy()
        gathered = [_S(r[:K], int(r[K])) for r in rows]

        def select(samples):
            args = _args(K, pbuffer_num=10 if K == 2 else 6, num_tasks=6, sparsity=0.5)
            pop = population.make_population(args)
            pop.update(samples)
            objs = np.array([s.objs for s in samples])
            ep = _EP([samples[i] for i in pareto.get_ep_indices(objs)])
            np.random.seed(7)
            el, sc, pr = pop.prediction_guided_selection(
                args, 0, ep, og, WeightedSumScalarization(num_objs=K, weights=np.ones(K) / K))
            return ([e.optgraph_id for e in el], np.array([s.weights.numpy() for s in sc]), np.array(pr))

        ids, w, pr = select(gathered)
        ids0, w0, pr0 = select(offspring)
        assert ids == ids0 and np.array_equal(w, w0) and np.array_equal(pr, pr0)
        pick = torch.tensor(np.concatenate([np.array(ids, dtype=np.float64), w.ravel(), pr.ravel()]))
        every = [torch.empty_like(pick) for _ in range(ws)]
        dist.all_gather(every, pick)
        assert all(torch.equal(every[0], t) for t in every)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surfaced by the parent
        errq.put(f'rank {rank}: {e!r}')
        raise


@pytest.mark.parametrize('ws,K', [(2, 2), (2, 3)])
def test_selection_agrees_across_ranks_gloo(ws, K):
    ctx = mp.get_context('spawn')
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_selection_worker, args=(r, ws, port, K, errq)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _spawn(target, ws, *args):
    ctx = mp.get_context('spawn')
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, ws, port) + args + (errq,)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _place_worker(rank, ws, port, P, errq):
    """MOPGPopulation.place / materialize over gloo with CPU tensors: the elites of the next generation
    (drawn from the previous generation's offspring, each owned by the rank that produced it) move to the
    ranks that train them; only moved snapshots are sent, and bytes scale with the moves, not with P."""
    try:
        import argparse
        from pgmorl_amd.mopg import MOPGPopulation
        from pgmorl_amd.sample import DeviceSnapshot, Sample
        from pgmorl_amd.shard import owner_of
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        dist.init_process_group('gloo', rank=rank, world_size=ws)
        rt = MOPGPopulation(argparse.Namespace(env_name='MO-Hopper-v2'), device='cpu')
        lay = rt.layout
        L = lay.total

        def content(p):  # what the offspring of task p holds: params | m | v
            return torch.arange(3 * L, dtype=torch.float32).reshape(3, L) + 1000.0 * p

        # previous generation's offspring: task p ran on owner_of(p); elsewhere a remote handle
        prev = []
        for p in range(P):
            own = owner_of(p, P, ws)
            if own == rank:
                c = content(p)
                snap = DeviceSnapshot(lay, c[0], c[1], c[2], 7, owner=own)
            else:
                snap = DeviceSnapshot.remote(lay, 7, own)
            prev.append(Sample.from_snapshot(snap, {}, objs=None))
        # next generation's elites (a deterministic reshuffle, identical on every rank)
        pick = [(3 * p + 1) % P for p in range(P)]
        elites = [Sample.copy_from(prev[q]) for q in pick]
        nbytes = rt.place(elites, [owner_of(p, P, ws) for p in range(P)])
        moves = [(owner_of(q, P, ws), owner_of(p, P, ws)) for p, q in enumerate(pick)]
        sent = [sum(1 for s, d in moves if s == r and s != d) for r in range(ws)]
        assert nbytes == (max(sent) * 3 * L * 4 if max(sent) else 0)
        for p, q in enumerate(pick):
            if owner_of(p, P, ws) == rank:
                assert torch.equal(elites[p].snapshot.stacked(), content(q)), (p, q)
        # final writer: every offspring onto rank 0
        rt.materialize(prev, dst=0)
        if rank == 0:
            for p in range(P):
                assert torch.equal(prev[p].snapshot.stacked(), content(p))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surfaced by the parent
        errq.put(f'rank {rank}: {e!r}')
        raise


@pytest.mark.parametrize('ws,P', [(2, 5), (2, 8), (3, 7)])
def test_place_moves_only_relocated_snapshots_gloo(ws, P):
    _spawn(_place_worker, ws, P)


def _failure_worker(rank, ws, port, failing, P, errq, kind='timeout'):
    """MOPGPopulation.check_generation over gloo: the rank(s) in ``failing`` saw an exchange timeout in their update
    (kind 'timeout') or wrong Adam step counts (kind 'steps'); every rank -- also one that owns no task of the
    generation (tb None) -- must raise (PGMError / RuntimeError) together and then still complete a collective
    (nobody is left blocked in one)."""
    try:
        import argparse
        from pgmorl_amd._lib import PGMError
        from pgmorl_amd.mopg import MOPGPopulation
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        dist.init_process_group('gloo', rank=rank, world_size=ws)

        class _TB:  # stands in for TaskBatch's sticky timeout flag
            def take_update_failed(self):
                return kind == 'timeout' and rank in failing

        lo, hi = task_block(P, rank, ws)
        rt = MOPGPopulation(argparse.Namespace(env_name='MO-Hopper-v2'), device='cpu')
        raised = False
        mismatch = f'rank {rank}: steps' if kind == 'steps' and rank in failing else None
        try:
            rt.check_generation(_TB() if hi > lo else None, mismatch)
        except PGMError:
            raised = kind == 'timeout'
        except RuntimeError:
            raised = kind == 'steps'
        assert raised == bool(failing), (rank, raised)
        dist.barrier()  # every rank got here: no one hangs in the check's collective
        dist.destroy_process_group()
        if raised:
            raise SystemExit(3)  # exits non-zero like the generation loop would
    except SystemExit:
        raise
    except Exception as e:  # surfaced by the parent
        errq.put(f'rank {rank}: {e!r}')
        raise


@pytest.mark.parametrize('ws,failing,P,kind', [(2, (1,), 4, 'timeout'), (3, (0,), 2, 'timeout'), (3, (), 5, 'timeout'),
                                             (2, (0, 1), 2, 'timeout'), (2, (1,), 4, 'steps'), (3, (2,), 7, 'steps')])
def test_update_failure_raises_on_every_rank_gloo(ws, failing, P, kind):
    ctx = mp.get_context('spawn')
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_failure_worker, args=(r, ws, port, failing, P, errq, kind)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    want = 3 if failing else 0
    assert all(p.exitcode == want for p in procs), [p.exitcode for p in procs]
