"""ctypes binding of libpgm.so (include/pgm_abi.h).

torch is imported first so that the HIP runtime torch ships (same soname libamdhip64.so.7)
is the one libpgm.so binds to: device pointers and streams are then shared.
There is no fallback: if the library is missing or fails to load, every op raises.
"""
import contextlib
import ctypes as C
import os

import torch  # noqa: F401  (must precede loading libpgm.so)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('PGM_LIB') or os.path.join(HERE, 'libpgm.so')
TEST_LIB_PATH = os.path.join(HERE, 'libpgm_test.so')  # -DPGM_TEST_HOOKS build (pgmorl_amd/build.py), tests only

PGM_ABI_VERSION = 4
PGM_OK, PGM_E_INVALID_ARG, PGM_E_SHAPE, PGM_E_HIP, PGM_E_UNSUPPORTED = 0, -1, -2, -3, -4
PARAM_TENSORS = ['actor_w1', 'actor_b1', 'actor_w2', 'actor_b2', 'critic_w1', 'critic_b1', 'critic_w2',
                 'critic_b2', 'value_w', 'value_b', 'mean_w', 'mean_b', 'logstd']

P_ = C.c_void_p
I32 = C.c_int32
F32 = C.c_float
F64 = C.c_double


class Dims(C.Structure):
    _fields_ = [(n, I32) for n in ('P', 'N', 'T', 'O', 'A', 'K', 'H')]


class EnvSpec(C.Structure):
    _fields_ = [('d', P_), ('U', P_), ('c', P_), ('V', P_), ('ebase', P_), ('ecoef', P_), ('act_lo', P_),
                ('act_hi', P_), ('max_episode_steps', I32), ('_pad', I32)]


class EnvState(C.Structure):
    _fields_ = [('s', P_), ('elapsed', P_), ('obj_acc', P_), ('obj_acc_valid', P_), ('ret', P_), ('s0', P_)]


class NormState(C.Structure):
    _fields_ = [('ob_mean', P_), ('ob_var', P_), ('ob_count', P_), ('ret_mean', P_), ('ret_var', P_),
                ('ret_count', P_), ('obj_mean', P_), ('obj_var', P_), ('obj_count', P_), ('gamma', F64),
                ('clipob', F64), ('cliprew', F64), ('epsilon', F64), ('use_ob_rms', I32), ('use_obj_rms', I32)]


class RolloutBuf(C.Structure):
    _fields_ = [(n, P_) for n in ('obs', 'actions', 'logp', 'values', 'rewards', 'masks', 'bad_masks',
                                  'returns', 'adv')]


class PPOHParams(C.Structure):
    _fields_ = [('clip_param', F32), ('value_loss_coef', F32), ('entropy_coef', F32), ('max_grad_norm', F32),
                ('adam_eps', F32), ('beta1', F32), ('beta2', F32), ('_pad', F32), ('ppo_epoch', I32),
                ('num_mini_batch', I32), ('use_clipped_value_loss', I32), ('_pad2', I32)]


class LaunchOpts(C.Structure):
    """pgm_launch_opts (pgm_abi.h): which kernel family an entry point may launch; all zero = automatic."""
    _fields_ = [(n, I32) for n in ('update_kernel', 'update_split', 'fs_one_per_cu', 'rollout_kernel', 'eval_kernel',
                                   '_pad')]


UPDATE_KERNELS = {'': 0, 'auto': 0, 'fs': 1, 'mfma': 2, 'rowsplit': 2, 'valu': 3}
UPDATE_SPLITS = {'': 0, '0': 1, '1': 2, '2': 3, '3': 3, '4': 4}  # the row-split cap -> PGM_SPLIT_*


def launch_opts(env=None):
    """The launch options of the A/B environment variables (read here, at every call: the library reads none):
    PGM_UPDATE_KERNEL = auto | fs | mfma | valu, PGM_UPDATE_SPLIT = 0 | 1 | 2 | 4 (row-split cap), PGM_FS_DUAL = 0
    (feature-split one workgroup per CU), PGM_ROLLOUT_KERNEL / PGM_EVAL_KERNEL = block."""
    env = os.environ if env is None else env
    k = env.get('PGM_UPDATE_KERNEL', '').strip().lower()
    sp = env.get('PGM_UPDATE_SPLIT', '').strip()
    if k not in UPDATE_KERNELS:
        raise PGMError(f'PGM_UPDATE_KERNEL={k!r}: expected one of {sorted(UPDATE_KERNELS)}')
    if sp not in UPDATE_SPLITS:
        raise PGMError(f'PGM_UPDATE_SPLIT={sp!r}: expected 0, 1, 2 or 4')
    return LaunchOpts(update_kernel=UPDATE_KERNELS[k], update_split=UPDATE_SPLITS[sp],
                      fs_one_per_cu=int(env.get('PGM_FS_DUAL', '').strip() == '0'),
                      rollout_kernel=int(env.get('PGM_ROLLOUT_KERNEL', '').strip().lower().startswith('b')),
                      eval_kernel=int(env.get('PGM_EVAL_KERNEL', '').strip().lower().startswith('b')))


_SIGS = {
    'pgm_abi_version': (C.c_int, []),
    'pgm_last_error': (C.c_char_p, []),
    'pgm_param_layout': (C.c_int, [I32, I32, I32, I32, C.POINTER(I32), C.POINTER(I32)]),
    'pgm_act_forward': (C.c_int, [C.POINTER(Dims), P_, P_, P_, I32, P_, P_, P_, P_]),
    'pgm_env_reset': (C.c_int, [C.POINTER(Dims), C.POINTER(EnvSpec), C.POINTER(EnvState), C.POINTER(NormState),
                                P_, P_]),
    'pgm_env_step': (C.c_int, [C.POINTER(Dims), C.POINTER(EnvSpec), C.POINTER(EnvState), C.POINTER(NormState),
                               P_, P_, P_, P_, P_, P_]),
    'pgm_rollout': (C.c_int, [C.POINTER(Dims), P_, C.POINTER(EnvSpec), C.POINTER(EnvState), C.POINTER(NormState),
                              C.POINTER(RolloutBuf), P_, C.c_uint64, I32, C.POINTER(LaunchOpts), P_]),
    'pgm_gae': (C.c_int, [C.POINTER(Dims), C.POINTER(RolloutBuf), F32, F32, I32, I32, P_]),
    'pgm_adv_normalize': (C.c_int, [C.POINTER(Dims), C.POINTER(RolloutBuf), P_, P_, P_]),
    'pgm_ppo_update': (C.c_int, [C.POINTER(Dims), C.POINTER(PPOHParams), P_, P_, P_, P_, P_, P_,
                                 C.POINTER(RolloutBuf), P_, P_, C.POINTER(LaunchOpts), P_]),
    'pgm_ppo_update_workspace_bytes': (C.c_size_t, [C.POINTER(Dims)]),
    'pgm_ppo_update_variant': (C.c_int, [C.POINTER(Dims), C.c_void_p, C.POINTER(LaunchOpts), C.c_char_p, C.c_int]),
    'pgm_ppo_update_reset': (C.c_int, [C.POINTER(Dims), P_, P_]),
    'pgm_ppo_fs_fragment_map': (C.c_int, [I32, I32, I32, I32, C.POINTER(I32), I32]),
    'pgm_eval': (C.c_int, [C.POINTER(Dims), P_, C.POINTER(EnvSpec), P_, P_, P_, I32, I32, I32, F64, P_,
                           C.POINTER(LaunchOpts), P_]),
    'pgm_randperm': (C.c_int, [I32, I32, C.c_uint64, P_, P_]),
    'pgm_normal_noise': (C.c_int, [C.c_int64, C.c_uint64, P_, P_]),
}

EXPORTS = tuple(_SIGS)

_libs = {}
_active = None


class PGMError(RuntimeError):
    pass


def _load(path):
    if path not in _libs:
        if not os.path.exists(path):
            raise PGMError(f'{path} not built; run `python -m pgmorl_amd.build` (hipcc, gfx950)')
        h = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            f = getattr(h, name)
            f.restype, f.argtypes = res, args
        if h.pgm_abi_version() != PGM_ABI_VERSION:
            raise PGMError(f'{path}: ABI {h.pgm_abi_version()} != {PGM_ABI_VERSION}')
        _libs[path] = h
    return _libs[path]


def lib():
    """The loaded libpgm.so (raises if it is missing: there is no CPU fallback); inside test_build(), the test
    build."""
    return _active if _active is not None else _load(LIB_PATH)


@contextlib.contextmanager
def test_build():
    """Route every call of the block through libpgm_test.so, the build with the PGM_TEST_DELAY /
    PGM_TEST_RESIDENT_CUS hooks (tests only; the production library has neither)."""
    global _active
    prev, _active = _active, _load(TEST_LIB_PATH)
    try:
        yield _active
    finally:
        _active = prev


def check(rc, what):
    if rc != PGM_OK:
        msg = lib().pgm_last_error().decode(errors='replace')
        raise PGMError(f'{what} failed ({rc}): {msg}')


def param_layout(O, A, K, H=64):
    """(offsets dict, total) of the flat per-task parameter vector (pgm_param_layout)."""
    offs = (I32 * 13)()
    tot = I32()
    check(lib().pgm_param_layout(O, A, K, H, offs, C.byref(tot)), 'pgm_param_layout')
    return dict(zip(PARAM_TENSORS, list(offs))), tot.value
