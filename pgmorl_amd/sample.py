"""Reference-compatible Sample / Task / WeightedSumScalarization / RunningMeanStd (host API).

A ``Sample`` (morl/sample.py:10-32) is a policy snapshot: env_params (running statistics),
actor_critic, agent (optimizer state), objs and optgraph_id.  In this build the policy and Adam
state of a snapshot stay in HBM (``DeviceSnapshot``, one row of a [P, L] device tensor captured
right after an iteration) and are only materialised as reference-format tensors on demand:
``sample.actor_critic.state_dict()`` gives the reference's state_dict (fp64, reference keys), and
``sample.agent.optimizer.state_dict()`` a torch Adam state_dict.
"""
import copy

import numpy as np
import torch


class RunningMeanStd:
    """Parallel-variance running statistics, same fields as baselines' RunningMeanStd
    (externals/baselines/baselines/common/running_mean_std.py:3-31)."""

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

    def update_weights(self, weights):
        if weights is not None:
            self.weights = torch.tensor(np.asarray(weights, dtype=np.float64))

    def update_z(self, z):
        pass

    def evaluate(self, objs):
        return (objs * self.weights).sum(axis=-1)


class DeviceSnapshot:
    """Parameters + Adam state of one task, kept on the device of the rank that produced it.

    Multi-GPU: every rank holds the same Samples (identical host state), but a snapshot's tensors live
    only on its ``owner`` rank; elsewhere it is a remote handle (``data is None``) that
    ``MOPGPopulation`` moves to the rank that next trains it, or to rank 0 for the final artefacts
    (shard.move_rows: bytes scale with the moved snapshots, not with the population).  owner None =
    local (single process, or replicated on every rank like the warm-up policies)."""

    def __init__(self, layout, params, adam_m, adam_v, adam_step, owner=None):
        self.layout = layout
        self.data = None if params is None else (params, adam_m, adam_v)
        self.adam_step = int(adam_step)
        self.owner = owner

    @classmethod
    def remote(cls, layout, adam_step, owner):
        return cls(layout, None, None, None, adam_step, owner)

    @property
    def is_local(self):
        return self.data is not None

    def _part(self, i):
        if self.data is None:
            raise RuntimeError(f'snapshot lives on rank {self.owner}: move it first (MOPGPopulation.materialize)')
        return self.data[i]

    params = property(lambda self: self._part(0))
    adam_m = property(lambda self: self._part(1))
    adam_v = property(lambda self: self._part(2))

    def stacked(self):
        """[3, L] params | exp_avg | exp_avg_sq (a new tensor)."""
        return torch.stack([self.params, self.adam_m, self.adam_v])

    def adopt(self, rows):
        """Materialise a remote handle from a received [3, L] block (it becomes local)."""
        self.data = (rows[0].clone(), rows[1].clone(), rows[2].clone())

    def clone(self):
        if self.data is None:
            return DeviceSnapshot.remote(self.layout, self.adam_step, self.owner)
        return DeviceSnapshot(self.layout, self.params.clone(), self.adam_m.clone(), self.adam_v.clone(),
                              self.adam_step, self.owner)


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
    def __init__(self, env_params, actor_critic, agent, objs=None, optgraph_id=None):
        self.env_params = env_params
        self.actor_critic = actor_critic
        self.agent = agent
        self.objs = objs
        self.optgraph_id = optgraph_id

    @property
    def snapshot(self):
        return self.actor_critic.snap

    @classmethod
    def from_snapshot(cls, snap, env_params, objs=None, optgraph_id=None):
        return cls(env_params, PolicyHandle(snap), AgentHandle(snap), objs, optgraph_id)

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
