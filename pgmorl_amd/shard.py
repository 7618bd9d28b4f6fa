"""Task sharding across GPUs and the generation-boundary exchange.

Tasks never interact inside a generation (morl/mopg.py:60-182 touches only its own task), so each
rank (one process per GPU) owns a contiguous block of ceil(P/G) tasks for the whole generation and the
data path has no collective.  At the generation boundary (morl/morl.py:90-125) only the fp64 RECORDS of
every offspring (objective vector, running statistics, Adam step) are all-gathered (``allgather_rows``,
a few KB), so every rank runs the identical host EP / OptGraph / selection.  Policy / Adam snapshots stay
on the rank that produced them and move point-to-multipoint (``move_rows``) only when a later generation
trains them on another rank, or when rank 0 writes the final EP policies.

Snapshot memory model: ``DeviceSnapshot.owner`` stays the PRODUCING rank for the snapshot's whole life.
A rank that receives a moved snapshot adopts it as an extra local replica (``DeviceSnapshot.adopt``);
the producer keeps its original, so a moved elite is live on two ranks until both Samples are dropped.
With the "nccl" backend (RCCL over xGMI on ROCm) the payloads stay in HBM; the same code runs on "gloo"
with CPU tensors (tests).
"""
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def task_block(P, rank, world_size):
    """[lo, hi) of the contiguous block of tasks owned by ``rank`` (ceil(P/G) per rank, last ones short)."""
    per = -(-P // world_size)
    lo = min(P, rank * per)
    return lo, min(P, lo + per)


def owner_of(p, P, world_size):
    """The rank whose task_block holds task p."""
    per = -(-P // world_size)
    return min(p // per, world_size - 1)


def allgather_rows(local, P, group=None):
    """Concatenate every rank's ``local`` rows ([P_local, ...], rank order) into [P, ...] on every rank.

    Ranks may own different row counts (task_block); rows are padded to ceil(P/G) for the collective.
    """
    rank, ws = (dist.get_rank(group), dist.get_world_size(group)) if group is not None else world()
    if ws == 1:
        return local
    per = -(-P // ws)
    lo, hi = task_block(P, rank, ws)
    if local.shape[0] != hi - lo:
        raise ValueError(f'rank {rank}: {local.shape[0]} rows, block is {hi - lo}')
    buf = local.new_zeros((per,) + tuple(local.shape[1:]))
    buf[:hi - lo] = local
    parts = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(parts, buf.contiguous(), group=group)
    return torch.cat([parts[r][:task_block(P, r, ws)[1] - task_block(P, r, ws)[0]] for r in range(ws)])


def allreduce_max(values, device):
    """Max over ranks of a few host floats (timing: the slowest rank defines the step time)."""
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if world()[1] > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t]


def move_rows(moves, local_rows, shape, dtype, device, group=None):
    """Collective point-to-multipoint move of fixed-shape rows (the elite snapshots whose next task runs on
    another rank, or the EP snapshots rank 0 writes out).

    ``moves``: [(src, dst)] per item, in an order identical on every rank; ``local_rows[k]`` is item k's
    tensor on its src rank.  Returns ({k: tensor} of the items whose dst is this rank, bytes each rank
    contributed).  One all-gather of [max items sent by one rank, *shape]: the payload scales with the moved
    rows, not with the population (items with src == dst or src < 0, i.e. replicated, are not sent)."""
    rank, ws = (dist.get_rank(group), dist.get_world_size(group)) if group is not None else world()
    live = [(k, s, d) for k, (s, d) in enumerate(moves) if s is not None and s >= 0 and s != d]
    if ws == 1 or not live:
        return {}, 0
    sends = [[] for _ in range(ws)]
    for k, s, d in live:
        sends[s].append(k)
    per = max(len(x) for x in sends)
    buf = torch.zeros((per,) + tuple(shape), dtype=dtype, device=device)
    for j, k in enumerate(sends[rank]):
        buf[j].copy_(local_rows[k])
    parts = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(parts, buf, group=group)
    got = {}
    for s in range(ws):
        for j, k in enumerate(sends[s]):
            if moves[k][1] == rank:
                got[k] = parts[s][j].clone()
    return got, buf.numel() * buf.element_size()


def any_rank(flag, device):
    """Collective: True on EVERY rank when ``flag`` is true on any rank (a failure one rank detected must end
    the generation on all ranks together, before anyone enters the next collective)."""
    return allreduce_max([1.0 if flag else 0.0], device)[0] > 0.0
