"""Reference-compatible Sample / Task / WeightedSumScalarization / RunningMeanStd (host API).

A ``Sample`` (morl/sample.py:10-32) is a policy snapshot: env_params (running statistics),
actor_critic, agent (optimizer state), objs and optgraph_id.  In this build the policy and Adam
state of a snapshot stay in HBM (``DeviceSnapshot``, one row of a [P, L] device tensor captured
right after an iteration) and are only materialised as reference-format tensors on demand:
``sample.actor_critic.state_dict()`` gives the reference's state_dict (fp64, reference keys), and
``sample.agent.optimizer.state_dict()`` a torch Adam state_dict.
"""
import copy
import weakref

import numpy as np
import torch


class RunningMeanStd:
    """Parallel-variance running statistics, same fields as baselines' RunningMeanStd
    (externals/baselines/baselines/common/running_mean_std.py:3-31)."""

    def __deepcopy__(self, memo):
        c = RunningMeanStd.__new__(RunningMeanStd)
        c.mean, c.var, c.count = np.copy(self.mean), np.copy(self.var), self.count
        return c

    def __init__(self, epsilon=1e-4, shape=()):
        self.mean = np.zeros(shape, 'float64')
        self.var = np.ones(shape, 'float64')
        self.count = epsilon

    def update(self, x):
        x = np.asarray(x, dtype=np.float64)
        bm, bv, n = x.mean(axis=0), x.var(axis=0), x.shape[0]
        delta = bm - self.mean
        tot = self.count + n
        self.mean = self.mean + delta * n / tot
        self.var = (self.var * self.count + bv * n + np.square(delta) * self.count * n / tot) / tot
        self.count = tot


class WeightedSumScalarization:
    """morl/scalarization_methods.py:21-29."""

    def __init__(self, num_objs, weights=None):
        self.num_objs = num_objs
        self.weights = None if weights is None else torch.tensor(np.asarray(weights, dtype=np.float64))

    def __deepcopy__(self, memo):  # the generic path deep-copies the tensor through its storage (slow)
        c = WeightedSumScalarization.__new__(WeightedSumScalarization)
        c.num_objs = self.num_objs
        c.weights = None if self.weights is None else self.weights.clone()
        return c

    def update_weights(self, weights):
        if weights is not None:
            self.weights = torch.tensor(np.asarray(weights, dtype=np.float64))

    def update_z(self, z):
        pass

    def evaluate(self, objs):
        return (objs * self.weights).sum(axis=-1)


class RowStore:
    """Device storage shared by snapshots: a generation's arena ([I][3][Pl][L], key (i, slot)) or a compact
    buffer ([S][3][L], key k).  Tracks the snapshots that point into it (weakly), so ``compact_snapshots`` can
    move the survivors out and let the storage go.  Every live store is in ``RowStore.live``."""
    live = weakref.WeakSet()

    def __init__(self, tensor, kind):
        assert kind in ('arena', 'compact')
        self.t, self.kind = tensor, kind
        self.snaps = weakref.WeakSet()
        RowStore.live.add(self)

    @property
    def rows(self):
        return self.t.shape[0] * self.t.shape[2] if self.kind == 'arena' else self.t.shape[0]

    def view(self, key):
        return self.t[key[0], :, key[1]] if self.kind == 'arena' else self.t[key]


def compact_snapshots(min_live_frac=0.5):
    """Move the snapshots that are still alive out of every finished generation arena (and out of compact
    buffers less than ``min_live_frac`` live) into one new compact [S][3][L] buffer per source, by one gather
    each, and rewire them; the old storage is freed once nothing else references it.  Called at every generation
    boundary by pgmorl_amd.morl.run after EP / population / selection, so device memory follows the surviving
    snapshots (EP + population + elites), not every iteration of every task of the run.  Returns (stores
    compacted, rows kept)."""
    n_st = n_rows = 0
    for st in list(RowStore.live):
        snaps = [s for s in list(st.snaps) if s._store is st]
        if not snaps:
            continue
        keys = sorted({s._key for s in snaps})
        if st.kind == 'compact' and len(keys) >= min_live_frac * st.rows:
            continue
        if st.kind == 'arena':
            i = torch.tensor([k[0] for k in keys], device=st.t.device)
            q = torch.tensor([k[1] for k in keys], device=st.t.device)
            new = st.t[i, :, q]  # advanced indexing on dims 0 and 2 -> [S][3][L], a fresh tensor
        else:
            new = st.t[torch.tensor(keys, device=st.t.device)]
        ns = RowStore(new, 'compact')
        where = {k: j for j, k in enumerate(keys)}
        for s in snaps:
            s._bind(ns, where[s._key])
        st.snaps = weakref.WeakSet()
        n_st += 1
        n_rows += len(keys)
    return n_st, n_rows


class DeviceSnapshot:
    """Parameters + Adam state of one task, kept on the device of the rank that produced it.

    Snapshots are IMMUTABLE once taken: the per-iteration copies of a generation live in one device arena
    ([iterations][3][tasks][L], ``MOPGPopulation.run``) and a snapshot is an index into it (``in_arena``), so
    taking, cloning (Task / Sample.copy_from) and dropping snapshots moves no bytes.  Tensors are views,
    created on first use.  At the generation boundary ``compact_snapshots`` moves the survivors into a compact
    buffer, so an arena does not outlive its generation because one of its snapshots survived.

    Multi-GPU: every rank holds the same Samples (identical host state), but a snapshot's tensors live
    only on its ``owner`` rank; elsewhere it is a remote handle (no data) that ``MOPGPopulation`` moves to the
    rank that next trains it, or to rank 0 for the final artefacts (shard.move_rows: bytes scale with the
    moved snapshots, not with the population).  owner None = local (single process, or replicated on every
    rank like the warm-up policies)."""

    def __init__(self, layout, params, adam_m, adam_v, adam_step, owner=None):
        self.layout = layout
        self._data = None if params is None else (params, adam_m, adam_v)
        self._store, self._key = None, None  # (RowStore, key) -- the block view is made on demand
        self._blk = None
        self.adam_step = int(adam_step)
        self.owner = owner

    @classmethod
    def remote(cls, layout, adam_step, owner):
        return cls(layout, None, None, None, adam_step, owner)

    @classmethod
    def in_arena(cls, layout, store, i, slot, adam_step, owner=None):
        """Snapshot = row (i, :, slot) of a generation's arena store (no copy)."""
        s = cls(layout, None, None, None, adam_step, owner)
        s._bind(store, (i, slot))
        return s

    def _bind(self, store, key):
        self._store, self._key = store, key
        self._blk = self._data = None  # cached views of the previous storage
        if store is not None:
            store.snaps.add(self)

    @property
    def is_local(self):
        return self._data is not None or self._store is not None or self._blk is not None

    def block(self):
        """[3, L] params | exp_avg | exp_avg_sq (a view when the snapshot lives in a store or was adopted)."""
        if self._blk is None:
            if self._store is not None:
                self._blk = self._store.view(self._key)
            elif self._data is not None:
                self._blk = torch.stack(self._data)
            else:
                raise RuntimeError(f'snapshot lives on rank {self.owner}: move it first (MOPGPopulation.materialize)')
        return self._blk

    @property
    def data(self):
        if self._data is None and (self._store is not None or self._blk is not None):
            b = self.block()
            self._data = (b[0], b[1], b[2])
        return self._data

    def _part(self, i):
        d = self.data
        if d is None:
            raise RuntimeError(f'snapshot lives on rank {self.owner}: move it first (MOPGPopulation.materialize)')
        return d[i]

    params = property(lambda self: self._part(0))
    adam_m = property(lambda self: self._part(1))
    adam_v = property(lambda self: self._part(2))

    def stacked(self):
        """[3, L] params | exp_avg | exp_avg_sq (read-only: snapshots are never written)."""
        return self.block()

    def adopt(self, rows):
        """Materialise a remote handle from a received [3, L] block (it becomes a local replica)."""
        self._bind(None, None)
        self._blk = rows

    def clone(self):
        """Snapshots are immutable: a clone shares the device storage (no copy)."""
        c = DeviceSnapshot(self.layout, None, None, None, self.adam_step, self.owner)
        if self._store is not None:
            c._bind(self._store, self._key)
        else:
            c._data, c._blk = self._data, self._blk
        return c


class PolicyHandle:
    """Stands in for the reference's actor_critic module of a Sample."""

    def __init__(self, snap):
        self.snap = snap

    def state_dict(self):
        return self.snap.layout.unflatten(self.snap.params)

    def parameters(self):
        return list(self.state_dict().values())


class _OptimizerView:
    def __init__(self, snap, lr):
        self.snap, self.lr = snap, lr

    def state_dict(self):
        s = self.snap
        st = s.layout.adam_to_optimizer_state(s.adam_m.cpu(), s.adam_v.cpu(), s.adam_step)
        return {'state': st, 'param_groups': [{'lr': self.lr, 'betas': (0.9, 0.999), 'eps': 1e-5, 'weight_decay': 0,
                                               'amsgrad': False, 'params': list(range(13))}]}


class AgentHandle:
    """Stands in for the reference's PPO agent of a Sample (its optimizer state)."""

    def __init__(self, snap, lr=3e-4):
        self.snap = snap
        self.optimizer = _OptimizerView(snap, lr)


class Sample:
    __slots__ = ('_env_params', '_envp_fn', '_snap', '_actor_critic', '_agent', 'objs', 'optgraph_id', '__dict__')

    def __init__(self, env_params, actor_critic, agent, objs=None, optgraph_id=None):
        self._env_params, self._envp_fn = env_params, None
        self._snap = None
        self._actor_critic, self._agent = actor_critic, agent
        self.objs = objs
        self.optgraph_id = optgraph_id

    # the policy / agent handles of a device snapshot are made on first access (most offspring never need them)
    @property
    def actor_critic(self):
        if self._actor_critic is None and self._snap is not None:
            self._actor_critic = PolicyHandle(self._snap)
        return self._actor_critic

    @actor_critic.setter
    def actor_critic(self, v):
        self._actor_critic = v

    @property
    def agent(self):
        if self._agent is None and self._snap is not None:
            self._agent = AgentHandle(self._snap)
        return self._agent

    @agent.setter
    def agent(self, v):
        self._agent = v

    @property
    def env_params(self):
        """{'ob_rms', 'ret_rms', 'obj_rms'} RunningMeanStd copies (morl/sample.py:12).  An offspring built by
        MOPGPopulation.run unpacks them from its host record on first access (most offspring never need them)."""
        if self._envp_fn is not None:
            self._env_params, self._envp_fn = self._envp_fn(), None
        return self._env_params

    @env_params.setter
    def env_params(self, value):
        self._env_params, self._envp_fn = value, None

    @property
    def snapshot(self):
        return self._snap if self._snap is not None else self.actor_critic.snap

    @classmethod
    def from_snapshot(cls, snap, env_params, objs=None, optgraph_id=None):
        s = cls(env_params, None, None, objs, optgraph_id)
        s._snap = snap
        return s

    @classmethod
    def lazy(cls, snap, env_params_fn, objs=None, optgraph_id=None):
        """A Sample whose env_params are built by env_params_fn() on first access."""
        s = cls(None, None, None, objs, optgraph_id)
        s._snap = snap
        s._envp_fn = env_params_fn
        return s

    @classmethod
    def from_reference(cls, ref_sample, layout, device='cuda'):
        """Adopt a reference Sample (morl/sample.py: actor_critic module, agent with a torch Adam,
        env_params dict) as a device-resident one: parameters and Adam state move to HBM in the
        flat layout, env_params / objs / optgraph_id are kept."""
        sd = ref_sample.actor_critic.state_dict()
        opt = ref_sample.agent.optimizer.state_dict().get('state', {})
        m, v, step = layout.adam_from_optimizer_state(opt)
        dev = torch.device(device)
        snap = DeviceSnapshot(layout, torch.from_numpy(layout.flatten(sd)).to(dev), torch.from_numpy(m).to(dev),
                              torch.from_numpy(v).to(dev), step)
        return cls.from_snapshot(snap, copy.deepcopy(ref_sample.env_params), copy.deepcopy(ref_sample.objs),
                                 ref_sample.optgraph_id)

    @classmethod
    def copy_from(cls, sample):
        snap = sample.snapshot.clone()
        return cls.from_snapshot(snap, copy.deepcopy(sample.env_params), copy.deepcopy(sample.objs),
                                 sample.optgraph_id)


class Task:
    """A (policy, weight) pair (morl/task.py:7-10)."""

    def __init__(self, sample, scalarization):
        self.sample = Sample.copy_from(sample)
        self.scalarization = copy.deepcopy(scalarization)
