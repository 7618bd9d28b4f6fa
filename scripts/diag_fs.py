"""Diagnostic: which parameter tensors of the feature-split update differ from the fp64 oracle, after 1 and 2 Adam
steps (test infrastructure: runs the oracle).

    PGM_UPDATE_KERNEL=fs python scripts/diag_fs.py MO-Hopper-v2 5 1 64
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ppo as oppo  # noqa: E402
from tests.test_gpu_kernels import _update_setup  # noqa: E402


def main():
    env, P, N, mb = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    for E, M in [(1, 1), (1, 2), (2, 2)]:
        T = mb * M // N
        args, spec, tb, pols, data, perms = _update_setup(env, P, T, N, E, M, seed=41)
        obs, actions, logp, values, returns, adv = data
        tb.lr.fill_(3e-4)
        tb.ppo_update(torch.stack(perms).numpy())
        tb.check_update()
        print(f'E={E} M={M} variant {tb.update_variant()}')
        params = tb.params.cpu().double().numpy()
        for p in range(min(P, 2)):
            agent = oppo.PPO(pols[p], args.clip_param, E, M, args.value_loss_coef, 0.0, lr=3e-4, eps=1e-5,
                             max_grad_norm=args.max_grad_norm)
            ro = oppo.RolloutStorage(T, N, spec['obs_dim'], spec['act_dim'], spec['obj_num'])
            ro.obs.copy_(torch.from_numpy(obs[p]).double())
            ro.actions.copy_(actions[p].double())
            ro.action_log_probs.copy_(logp[p].double().unsqueeze(-1))
            ro.value_preds.copy_(values[p].double())
            ro.returns.copy_(returns[p].double())
            for e in range(E):
                for mbt in ro.minibatches(adv[p].double(), M, perms[e]):
                    agent.minibatch_step(*mbt)
            ref = tb.layout.flatten(pols[p].state_dict(), dtype=np.float64)
            offs = sorted(tb.layout.offsets.items(), key=lambda kv: kv[1])
            for i, (name, off) in enumerate(offs):
                end = offs[i + 1][1] if i + 1 < len(offs) else tb.layout.total
                a, b = params[p, off:end], ref[off:end]
                err = np.abs(a - b)
                bad = err > 2e-6 + 1e-5 * np.abs(b)
                print(f'  task {p} {name:12s} n={end - off:5d} off={bad.sum():5d} max={err.max():.2e}')

if __name__ == '__main__':
    main()
