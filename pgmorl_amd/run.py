"""Entry point with the reference's flags and defaults (morl/run.py:52-93, morl/arguments.py:3-173).

    python -m pgmorl_amd.run --env-name MO-Walker2d-v2 --num-env-steps 5000000 ... [--selection-method ra]

Adds ``--rng {device,host}`` (device counter streams, or the reference's own torch draws for
bit-compatible runs) and ``--device``.
"""
import argparse
import os
import sys

import torch

DEFAULTS = ['--lr', '3e-4', '--use-linear-lr-decay', '--gamma', '0.995', '--use-gae', '--gae-lambda', '0.95',
            '--entropy-coef', '0', '--value-loss-coef', '0.5', '--num-steps', '2048', '--num-processes', '4',
            '--ppo-epoch', '10', '--num-mini-batch', '32', '--use-proper-time-limits', '--ob-rms', '--obj-rms',
            '--raw']


def get_parser():
    ap = argparse.ArgumentParser(description='PG-MORL on MI355X')
    add = ap.add_argument
    add('--env-name', default='MO-HalfCheetah-v2')
    add('--obj-num', type=int, default=2)
    add('--num-env-steps', type=int, default=5e6)
    add('--num-tasks', type=int, default=6)
    add('--seed', type=int, default=0)
    add('--min-weight', type=float, default=0.0)
    add('--max-weight', type=float, default=1.0)
    add('--delta-weight', type=float, default=0.2)
    add('--warmup-iter', type=int, default=80)
    add('--update-iter', type=int, default=20)
    add('--eval-num', type=int, default=1)
    add('--selection-method', type=str, default='prediction-guided')
    add('--pbuffer-num', type=int, default=100)
    add('--pbuffer-size', type=int, default=2)
    add('--num-weight-candidates', type=int, default=7)
    add('--sparsity', type=float, default=1.0)
    add('--obj-rms', default=False, action='store_true')
    add('--ob-rms', default=False, action='store_true')
    add('--raw', default=False, action='store_true')
    add('--rl-log-interval', type=int, default=10)
    add('--save-dir', default='./trained_models/')
    add('--algo', default='ppo')
    add('--lr', type=float, default=3e-4)
    add('--use-linear-lr-decay', action='store_true', default=False)
    add('--lr-decay-ratio', type=float, default=1.0)
    add('--gamma', type=float, default=0.995)
    add('--use-gae', action='store_true', default=False)
    add('--gae-lambda', type=float, default=0.95)
    add('--entropy-coef', type=float, default=0.0)
    add('--value-loss-coef', type=float, default=0.5)
    add('--max-grad-norm', type=float, default=0.5)
    add('--num-steps', type=int, default=2048)
    add('--num-processes', type=int, default=4)
    add('--ppo-epoch', type=int, default=10)
    add('--num-mini-batch', type=int, default=32)
    add('--clip-param', type=float, default=0.2)
    add('--use-proper-time-limits', action='store_true', default=False)
    add('--layernorm', action='store_true', default=False)
    add('--rng', choices=['device', 'host'], default='device')
    add('--device', default='cuda')
    return ap


def merge_argv(argv):
    """Command-line flags override the defaults (morl/run.py:29-50)."""
    defaults = list(DEFAULTS)
    for a in argv:
        if a.startswith('-') and a in defaults:
            i = defaults.index(a)
            j = i + 1
            while j < len(defaults) and not defaults[j].startswith('-'):
                j += 1
            del defaults[i:j]
    return defaults + list(argv)


class _Tee:
    def __init__(self, stream, f):
        self.stream, self.f = stream, f

    def write(self, d):
        self.stream.write(d)
        self.stream.flush()
        self.f.write(d)

    def flush(self):
        pass


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    torch.set_default_dtype(torch.float64)
    args = get_parser().parse_args(merge_argv(argv))
    if args.layernorm:
        raise NotImplementedError('--layernorm towers are not implemented by the MI355X kernels')
    os.makedirs(args.save_dir, exist_ok=True)
    with open(os.path.join(args.save_dir, 'args.txt'), 'w') as fp:
        fp.write(str(merge_argv(argv)))
    from .morl import run
    with open(os.path.join(args.save_dir, 'log.txt'), 'w') as logf:
        tee = _Tee(sys.stdout, logf)
        run(args, device=args.device, rng=args.rng, log=lambda *m: tee.write(' '.join(str(x) for x in m) + '\n'))


if __name__ == '__main__':
    main()
