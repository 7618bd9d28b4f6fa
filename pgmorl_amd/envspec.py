"""SynthMO environment specifications (the build's MuJoCo replacement).

MuJoCo is absent here and on the GPU box, so every MO-* env id of the reference
(environments/__init__.py:3-43) maps to a synthetic env with the same
(obs_dim, act_dim, obj_num, episode length) and an objective of the same form
as the reference env's ``step`` (environments/walker2d.py:16-30 etc.):

    a_c  = clip(a, act_lo, act_hi)
    s'   = tanh(d * s + U @ a_c + c)                      (obs = s')
    obj  = V @ s' + ebase - ecoef * sum(a_c ** 2)         ([K])

Episodes are fixed-length (done only at the time limit, so bad_transition is
always set, a2c_ppo_acktr/envs.py:125-126).  Constants come from splitmix64
(seed 1234) and are pinned by committed fixtures (tests/golden/synth_env_*.npz).
Reset states s0 are drawn per env seed (``args.seed + rank``) from splitmix64.
"""
import numpy as np

_M64 = (1 << 64) - 1


def _splitmix64_stream(seed):
    x = seed & _M64
    while True:
        x = (x + 0x9E3779B97F4A7C15) & _M64
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        yield z ^ (z >> 31)


def _uniforms(seed, n):
    g = _splitmix64_stream(seed)
    return np.array([(next(g) >> 11) * (1.0 / (1 << 53)) for _ in range(n)], dtype=np.float64)


# env id -> (obs_dim, act_dim, obj_num, max_episode_steps, action clip, objective coefficients)
#   obj rows: (velocity-like linear term scale, ebase, ecoef); scale 0 => no state term
_ENVS = {
    # walker2d.py:23-25: speed = v + 1, energy = 4 - sum(a^2) + 1
    'MO-Walker2d-v2': (17, 6, 2, 500, ([-1.0] * 6, [1.0] * 6), [(1.0, 1.0, 0.0), (0.0, 5.0, 1.0)]),
    # half_cheetah.py: run = min(4, v) + 1, energy = 5 - sum(a^2)
    'MO-HalfCheetah-v2': (17, 6, 2, 500, ([-1.0] * 6, [1.0] * 6), [(1.0, 1.0, 0.0), (0.0, 5.0, 1.0)]),
    # hopper.py: run/jump + alive - 2e-4 sum(a^2), clip [2,2,4]
    'MO-Hopper-v2': (11, 3, 2, 500, ([-2.0, -2.0, -4.0], [2.0, 2.0, 4.0]), [(1.5, 1.0, 2e-4), (1.0, 1.0, 2e-4)]),
    # hopper_v3.py: run, jump, energy
    'MO-Hopper-v3': (11, 3, 3, 500, ([-2.0, -2.0, -4.0], [2.0, 2.0, 4.0]),
                     [(1.5, 1.0, 0.0), (1.0, 1.0, 0.0), (0.0, 5.0, 1.0)]),
    # humanoid.py:33-35: run = 1.25 v + 3, energy = 3 - 4 sum(ctrl^2) + 3 (ctrlrange 0.4)
    'MO-Humanoid-v2': (376, 17, 2, 1000, ([-0.4] * 17, [0.4] * 17), [(1.25, 3.0, 0.0), (0.0, 6.0, 4.0)]),
    'MO-Ant-v2': (27, 8, 2, 500, ([-1.0] * 8, [1.0] * 8), [(1.0, 1.0, 0.0), (0.0, 5.0, 0.5)]),
    'MO-Swimmer-v2': (8, 2, 2, 500, ([-1.0] * 2, [1.0] * 2), [(1.0, 0.0, 0.0), (0.0, 0.3, 0.15)]),
}

SPEC_SEED = 1234


def env_names():
    return sorted(_ENVS)


def make_spec(env_name):
    """Constant arrays of one SynthMO env (all fp64)."""
    if env_name not in _ENVS:
        raise ValueError(f'unknown env {env_name!r}; known: {env_names()}')
    O, A, K, tmax, (lo, hi), objrows = _ENVS[env_name]
    u = _uniforms(SPEC_SEED, O + O * A + O + K * O)
    p = 0
    d = (2.0 * u[p:p + O] - 1.0) * 0.9; p += O
    U = ((2.0 * u[p:p + O * A] - 1.0) / np.sqrt(A)).reshape(O, A); p += O * A
    c = (2.0 * u[p:p + O] - 1.0) * 0.1; p += O
    V = np.zeros((K, O))
    for k, (scale, _, _) in enumerate(objrows):
        V[k] = (2.0 * u[p:p + O] - 1.0) * (2.0 * scale / np.sqrt(O))
        p += O
    return {
        'name': env_name, 'obs_dim': O, 'act_dim': A, 'obj_num': K, 'max_episode_steps': tmax,
        'd': d, 'U': U, 'c': c, 'V': V,
        'ebase': np.array([r[1] for r in objrows], dtype=np.float64),
        'ecoef': np.array([r[2] for r in objrows], dtype=np.float64),
        'act_lo': np.array(lo, dtype=np.float64), 'act_hi': np.array(hi, dtype=np.float64),
    }


def reset_state(obs_dim, env_seed):
    """Deterministic reset state of the env seeded ``env_seed`` (never the zero vector)."""
    return 0.5 * (2.0 * _uniforms(0x5EED0000 + int(env_seed), obs_dim) - 1.0)


def reset_table(obs_dim, seed, count):
    """s0 rows for env seeds seed+0 .. seed+count-1 (make_env seeds env rank with seed+rank)."""
    return np.stack([reset_state(obs_dim, seed + r) for r in range(count)])
