"""Debug: wide rollout vs block kernel vs oracle (Humanoid), per-step max obs error."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
from tests.test_gpu_kernels import _batch_with_policies, _oracle_rollout
from oracle import ppo as oppo
from oracle.vecenv import VecNormalizedSynth
from pgmorl_amd import envspec
env, N, T, P = 'MO-Humanoid-v2', int(sys.argv[1]) if len(sys.argv) > 1 else 8, 12, 1
res = {}
for kern in ('lanes', 'block'):
    os.environ['PGM_ROLLOUT_KERNEL'] = kern
    spec, tb, pols = _batch_with_policies(env, P, N, T, seed=3, scale=0.05)
    noise = torch.randn(T, N, spec['act_dim'], generator=torch.Generator().manual_seed(4), dtype=torch.float64)
    tb.env_reset()
    obs0 = tb.obs[0, 0].cpu().numpy().copy()
    tb.rollout(0, noise=noise.float(), carry=False)
    res[kern] = {k: getattr(tb, k)[0].cpu().numpy().copy() for k in ('obs', 'actions', 'logp', 'rewards')}
    res[kern]['obs0'] = obs0
s0 = envspec.reset_table(spec['obs_dim'], 0, N)
envs = VecNormalizedSynth(spec, s0, 0.995)
ro = oppo.RolloutStorage(T, N, spec['obs_dim'], spec['act_dim'], spec['obj_num'])
ro.obs[0].copy_(torch.from_numpy(envs.reset()).double())
_oracle_rollout(pols[0], envs, ro, noise.float().double())
ref = {'obs': ro.obs.numpy(), 'actions': ro.actions.numpy(), 'logp': ro.action_log_probs[..., 0].numpy(),
       'rewards': ro.rewards.numpy()}
for kern in res:
    print(kern, 'obs0 err', np.abs(res[kern]['obs0'] - ref['obs'][0]).max())
    for t in range(T):
        print(kern, t, 'obs', np.abs(res[kern]['obs'][t + 1] - ref['obs'][t + 1]).max(),
              'act', np.abs(res[kern]['actions'][t] - ref['actions'][t]).max(),
              'logp', np.abs(res[kern]['logp'][t] - ref['logp'][t]).max(),
              'rew', np.abs(res[kern]['rewards'][t] - ref['rewards'][t]).max())
    e = np.abs(res[kern]['obs'][1] - ref['obs'][1])
    idx = np.argwhere(e > 1e-4)
    print(kern, 'step1 bad (env, feature) first 20:', idx[:20].tolist(), len(idx))
