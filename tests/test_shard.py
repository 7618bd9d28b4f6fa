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

