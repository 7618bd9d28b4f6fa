"""Host-side profile of the whole generation loop on CPU (no GPU): pgmorl_amd.morl.run with a stand-in MOPG back end
whose offspring drift along their task weight (objectives only; parameters are a shared CPU arena).  Everything
else -- Tasks, offspring Samples, EP / population / OptGraph, prediction-guided selection, the writer thread and
the final EP files -- is the real code.  Usage: python scripts/prof_host.py [gens] [--profile]"""
import argparse
import cProfile
import os
import pstats
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pgmorl_amd.layout import ParamLayout  # noqa: E402
from pgmorl_amd.morl import run as morl_run  # noqa: E402
from pgmorl_amd.run import get_parser, merge_argv  # noqa: E402
from pgmorl_amd.sample import DeviceSnapshot, RowStore, RunningMeanStd, Sample  # noqa: E402


class StandIn:
    def __init__(self, args):
        self.args, self.device = args, torch.device('cpu')
        self.lay = ParamLayout(17, 6, 2)
        self.rng = np.random.RandomState(0)

    @property
    def layout(self):
        return self.lay

    def _batch(self, P):
        return self

    def evaluate_samples(self, samples, weights):
        return np.array([200 + 50 * self.rng.rand(2) for _ in samples])

    def materialize(self, samples, dst=0):
        return 0

    def run(self, task_batch, iteration, num_updates, start_time=None, log=None):
        a = self.args
        total = int(a.num_env_steps) // a.num_steps // a.num_processes
        I = len(range(iteration, min(iteration + num_updates, total)))
        P = len(task_batch)
        arena = RowStore(torch.zeros(I, 3, P, self.lay.total), 'arena')
        out = []
        for p, t in enumerate(task_batch):
            w = t.scalarization.weights.numpy()
            objs = np.asarray(t.sample.objs, dtype=np.float64)
            offs = []
            for i in range(I):
                objs = objs + 2.0 * w * self.rng.rand() + 0.5 * self.rng.randn(2)
                snap = DeviceSnapshot.in_arena(self.lay, arena, i, p, t.sample.snapshot.adam_step + 320 * (i + 1))
                offs.append(Sample.lazy(snap, lambda: {'ob_rms': RunningMeanStd(shape=(17,)), 'ret_rms': RunningMeanStd(),
                                                      'obj_rms': RunningMeanStd(shape=(2,))}, objs.copy()))
            out.append(offs)
        return out


def main():
    gens = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 26
    save = tempfile.mkdtemp(prefix='pgm_host_')
    argv = ['--env-name', 'MO-Walker2d-v2', '--obj-num', '2', '--num-env-steps', str((80 + 20 * gens) * 8192),
            '--warmup-iter', '80', '--update-iter', '20', '--delta-weight', repr(1.0 / 39), '--pbuffer-num', '100',
            '--pbuffer-size', '2', '--selection-method', 'prediction-guided', '--num-weight-candidates', '7',
            '--num-tasks', '40', '--sparsity', '1.0', '--obj-rms', '--ob-rms', '--raw', '--save-dir', save]
    torch.set_default_dtype(torch.float64)
    args = get_parser().parse_args(merge_argv(argv))
    rt = StandIn(args)
    pr = cProfile.Profile() if '--profile' in sys.argv else None
    t0 = time.perf_counter()
    if pr:
        pr.enable()
    ep = morl_run(args, device='cpu', log=None, runtime=rt)
    if pr:
        pr.disable()
    tm = ep.timing
    print(f"wall {time.perf_counter() - t0:.2f} s: host boundary {tm['host_s']:.3f} s over {len(tm['generations'])} "
          f"generations, stand-in MOPG {tm['rl_s']:.3f} s, final {tm.get('final_s', 0):.3f} s, EP {len(ep.obj_batch)}")
    if pr:
        pstats.Stats(pr).sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
