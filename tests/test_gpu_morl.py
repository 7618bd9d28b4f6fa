"""The host drop-in end to end on the device: pgmorl_amd.morl.run (warm-up + evolutionary generations with
MOPGPopulation in place of the per-task process fan-out) writes the reference's results/ tree."""
import os

import numpy as np
import pytest
import torch

from pgmorl_amd import pareto
from pgmorl_amd.layout import STATE_KEYS
from pgmorl_amd.morl import run
from pgmorl_amd.run import get_parser, merge_argv

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('env,K,selection', [('MO-Hopper-v2', 2, 'prediction-guided'), ('MO-Hopper-v2', 2, 'random'),
                                             ('MO-Hopper-v2', 2, 'ra'), ('MO-Hopper-v2', 2, 'moead'),
                                             ('MO-Hopper-v3', 3, 'prediction-guided')])
def test_morl_run_results_tree(gpu, tmp_path, env, K, selection):
    T, N = 32, 2
    argv = ['--env-name', env, '--obj-num', str(K), '--num-steps', str(T), '--num-processes', str(N), '--ppo-epoch', '1',
            '--num-mini-batch', '2', '--num-env-steps', str(T * N * 4), '--warmup-iter', '2', '--update-iter', '1',
            '--delta-weight', '0.5', '--selection-method', selection, '--save-dir', str(tmp_path),
            '--rl-log-interval', '1', '--rng', 'host', '--pbuffer-num', '100' if K == 2 else '5']
    args = get_parser().parse_args(merge_argv(argv))
    lines = []
    ep = run(args, device='cuda', rng='host', log=lines.append)
    assert any('[RL] Updates' in x for x in lines)
    for it in ('2', '3', '4'):
        for f in ('ep/objs.txt', 'population/objs.txt', 'population/optgraph.txt', 'elites/elites.txt',
                  'elites/weights.txt', 'elites/offsprings.txt'):
            assert os.path.exists(tmp_path / it / f), f'{it}/{f}'
        if selection == 'prediction-guided':
            pred = np.loadtxt(tmp_path / it / 'elites' / 'predictions.txt', delimiter=',', ndmin=2)
            assert pred.shape[1] == K and np.isfinite(pred).all()
    final = np.loadtxt(tmp_path / 'final' / 'objs.txt', delimiter=',', ndmin=2)
    assert final.shape == (len(ep.sample_batch), K)
    assert len(final) >= 1 and np.isfinite(final).all()
    np.testing.assert_allclose(final, ep.obj_batch, atol=1e-5)  # '{:5f}' text format of the archive
    assert list(pareto.get_ep_indices(ep.obj_batch)) == list(range(len(ep.obj_batch)))  # its own Pareto set
    offs = np.loadtxt(tmp_path / '2' / 'elites' / 'offsprings.txt', delimiter=',', ndmin=2)
    n_warm = len(pareto.weight_grid(K, 0.5))
    assert offs.shape == (n_warm * 2, K) and np.isfinite(offs).all()  # warm-up tasks x 2 warm-up iterations
    # every survivor was moved out of its generation's arena (device memory follows the survivors)
    from pgmorl_amd.sample import RowStore
    assert all(s.snapshot._store is None or s.snapshot._store.kind == 'compact' for s in ep.sample_batch)
    assert not [st for st in RowStore.live if st.kind == 'arena' and len(st.snaps)]
    sd = torch.load(tmp_path / 'final' / 'EP_policy_0.pt', weights_only=True)
    assert sorted(sd) == sorted(k for k, _, _ in STATE_KEYS)
    assert sd['dist.logstd._bias'].shape == (3, 1) and sd['base.actor.0.weight'].dtype == torch.float64
