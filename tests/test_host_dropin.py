"""Host side of the drop-in on CPU: reference Sample <-> device-layout Sample round trip, Task copies,
scalarisation, and the snapshot record packing used at the generation boundary."""
import argparse

import numpy as np
import torch

from oracle.mopg import initial_sample
from pgmorl_amd import envspec
from pgmorl_amd.layout import ParamLayout, STATE_KEYS
from pgmorl_amd.mopg import MOPGPopulation, host_draws, linear_lr
from pgmorl_amd.sample import Sample, Task, WeightedSumScalarization

from .helpers import small_args


def _trained_reference_sample():
    args = small_args('MO-Walker2d-v2')
    spec = envspec.make_spec('MO-Walker2d-v2')
    torch.manual_seed(3)
    s = initial_sample(args, spec)
    x = torch.randn(64, spec['obs_dim'], dtype=torch.float64)
    loss = s.actor_critic.get_value(x).pow(2).mean() + s.actor_critic.act(x)[2].mean()
    loss.backward()
    s.agent.optimizer.step()
    s.objs = np.array([1.5, -0.25])
    return s, spec


def test_from_reference_roundtrip():
    ref, spec = _trained_reference_sample()
    lay = ParamLayout(spec['obs_dim'], spec['act_dim'], spec['obj_num'])
    dev = Sample.from_reference(ref, lay, device='cpu')
    sd, want = dev.actor_critic.state_dict(), ref.actor_critic.state_dict()
    assert list(sd) == [k for k, _, _ in STATE_KEYS]
    for k in want:
        assert sd[k].shape == want[k].shape and sd[k].dtype == torch.float64
        torch.testing.assert_close(sd[k], want[k].float().double(), rtol=0, atol=0)
    st = dev.agent.optimizer.state_dict()['state']
    ref_st = ref.agent.optimizer.state_dict()['state']
    for i in ref_st:
        torch.testing.assert_close(st[i]['exp_avg'], ref_st[i]['exp_avg'].float().double(), rtol=0, atol=0)
        assert float(st[i]['step']) == float(ref_st[i]['step'])
    np.testing.assert_array_equal(dev.objs, ref.objs)
    # Task deep-copies its elite (morl/task.py:9-10): mutating the task's snapshot leaves the elite alone
    task = Task(dev, WeightedSumScalarization(2, [0.3, 0.7]))
    task.sample.snapshot.params.add_(1.0)
    assert not torch.equal(task.sample.snapshot.params, dev.snapshot.params)
    assert float(task.scalarization.evaluate(torch.tensor([2.0, 4.0]))) == 0.3 * 2.0 + 0.7 * 4.0


def test_record_unpack_matches_fields():
    args = argparse.Namespace(ob_rms=True, obj_rms=True)
    pop = MOPGPopulation.__new__(MOPGPopulation)
    pop.args = args
    O, K = 3, 2
    rec = np.arange(3 * K + 2 * O + 6, dtype=np.float64)
    objs, ep, step = pop._unpack(rec, O, K)
    np.testing.assert_array_equal(objs, [0, 1])
    np.testing.assert_array_equal(ep['ob_rms'].mean, [2, 3, 4])
    np.testing.assert_array_equal(ep['ob_rms'].var, [5, 6, 7])
    assert ep['ob_rms'].count == 8 and float(ep['ret_rms'].mean) == 9 and ep['ret_rms'].count == 11
    np.testing.assert_array_equal(ep['obj_rms'].mean, [12, 13])
    np.testing.assert_array_equal(ep['obj_rms'].var, [14, 15])
    assert ep['obj_rms'].count == 16 and step == 17


def test_host_draws_and_lr_schedule():
    z, perms = host_draws(5, 8, 2, 3, 2)
    torch.manual_seed(5)
    want = torch.stack([torch.normal(torch.zeros(2, 3, dtype=torch.float64), torch.ones(2, 3, dtype=torch.float64))
                        for _ in range(8)])
    torch.testing.assert_close(z, want.float(), rtol=0, atol=0)
    assert perms.shape == (2, 16) and sorted(perms[0].tolist()) == list(range(16))
    assert linear_lr(0, 100, 3e-4) == 3e-4 and abs(linear_lr(50, 100, 3e-4) - 1.5e-4) < 1e-18
