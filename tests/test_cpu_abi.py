"""CPU-side checks of the C ABI library: it loads, exports exactly what include/pgm_abi.h declares,
its structs match ctypes, and the parameter layout round-trips reference state_dicts.
No kernel is launched here (no GPU in this container)."""
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest
import torch

from pgmorl_amd import _lib
from pgmorl_amd.layout import STATE_KEYS, ParamLayout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'pgm_abi.h')


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(pgm_[a-z0-9_]+)\s*\(', src)))


def test_library_loads_and_reports_abi():
    assert _lib.lib().pgm_abi_version() == _lib.PGM_ABI_VERSION


def test_exports_every_declared_symbol():
    declared = _declared_functions()
    assert set(declared) == set(_lib.EXPORTS), (declared, _lib.EXPORTS)
    out = subprocess.run(['nm', '-D', '--defined-only', _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r' T (pgm_[a-z0-9_]+)', out))
    missing = set(declared) - exported
    assert not missing, missing


def test_struct_sizes_match_header():
    import ctypes as C
    prog = r'''
#include <stdio.h>
#include "pgm_abi.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(pgm_dims), sizeof(pgm_env_spec), sizeof(pgm_env_state),
         sizeof(pgm_norm_state), sizeof(pgm_rollout_buf), sizeof(pgm_ppo_hparams), sizeof(pgm_launch_opts));
  return 0; }
'''
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, 's.c'), os.path.join(d, 's')
        open(c, 'w').write(prog)
        subprocess.run(['gcc', '-I', os.path.join(ROOT, 'include'), c, '-o', exe], check=True)
        sizes = [int(x) for x in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    want = [C.sizeof(s) for s in (_lib.Dims, _lib.EnvSpec, _lib.EnvState, _lib.NormState, _lib.RolloutBuf,
                                   _lib.PPOHParams, _lib.LaunchOpts)]
    assert sizes == want


def test_production_library_reads_no_environment():
    """ABI 4: every launch choice is a pgm_launch_opts argument.  The production libpgm.so imports no getenv (the
    test hooks live only in libpgm_test.so, built -DPGM_TEST_HOOKS), and no source under csrc/ calls getenv outside
    a PGM_TEST_HOOKS block."""
    und = subprocess.run(['nm', '-D', '--undefined-only', _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert 'getenv' not in und
    if os.path.exists(_lib.TEST_LIB_PATH):
        und_t = subprocess.run(['nm', '-D', '--undefined-only', _lib.TEST_LIB_PATH], capture_output=True,
                               text=True).stdout
        assert 'getenv' in und_t  # the hooks are really in the test build
    csrc = os.path.join(ROOT, 'pgmorl_amd', 'csrc')
    for f in sorted(os.listdir(csrc)):
        depth, hooked = 0, []
        for i, line in enumerate(open(os.path.join(csrc, f)), 1):
            t = line.strip()
            if t.startswith('#if'):
                hooked.append('PGM_TEST_HOOKS' in t)
            elif t.startswith('#endif') and hooked:
                hooked.pop()
            if 'getenv' in line.split('//')[0]:
                assert any(hooked), f'{f}:{i} calls getenv outside #ifdef PGM_TEST_HOOKS'


def test_launch_opts_from_environment():
    o = _lib.launch_opts({})
    assert (o.update_kernel, o.update_split, o.fs_one_per_cu, o.rollout_kernel, o.eval_kernel) == (0, 0, 0, 0, 0)
    o = _lib.launch_opts({'PGM_UPDATE_KERNEL': 'fs', 'PGM_FS_DUAL': '0', 'PGM_ROLLOUT_KERNEL': 'block'})
    assert (o.update_kernel, o.fs_one_per_cu, o.rollout_kernel, o.eval_kernel) == (1, 1, 1, 0)
    for sp, want in (('0', 1), ('1', 2), ('2', 3), ('4', 4)):
        assert _lib.launch_opts({'PGM_UPDATE_SPLIT': sp, 'PGM_UPDATE_KERNEL': 'mfma'}).update_split == want
    assert _lib.launch_opts({'PGM_UPDATE_KERNEL': 'valu', 'PGM_EVAL_KERNEL': 'block'}).eval_kernel == 1
    with pytest.raises(_lib.PGMError):
        _lib.launch_opts({'PGM_UPDATE_KERNEL': 'bogus'})
    with pytest.raises(_lib.PGMError):
        _lib.launch_opts({'PGM_UPDATE_SPLIT': '7'})


def test_invalid_launch_opts_are_rejected_before_any_launch():
    import ctypes as C
    L = _lib.lib()
    d = _lib.Dims(2, 4, 64, 17, 6, 2, 64)
    hp = _lib.PPOHParams(0.2, 0.5, 0.0, 0.5, 1e-5, 0.9, 0.999, 0.0, 1, 2, 1, 0)
    buf = C.create_string_buffer(128)
    for bad in (_lib.LaunchOpts(update_kernel=9), _lib.LaunchOpts(update_split=-1), _lib.LaunchOpts(fs_one_per_cu=2),
                _lib.LaunchOpts(rollout_kernel=3), _lib.LaunchOpts(eval_kernel=-1)):
        assert L.pgm_ppo_update_variant(C.byref(d), C.byref(hp), C.byref(bad), buf, 128) == _lib.PGM_E_INVALID_ARG
        assert b'pgm_launch_opts' in L.pgm_last_error()
    # the VALU A/B choice is decided before any device query
    valu = _lib.LaunchOpts(update_kernel=3)
    assert L.pgm_ppo_update_variant(C.byref(d), C.byref(hp), C.byref(valu), buf, 128) == _lib.PGM_OK
    assert buf.value == b'ppo_update_kernel (VALU, A/B)'


def test_error_reporting_without_gpu():
    import ctypes as C
    L = _lib.lib()
    d = _lib.Dims(0, 4, 8, 17, 6, 2, 64)  # P=0 is rejected before any HIP call
    rc = L.pgm_gae(C.byref(d), None, 0.99, 0.95, 1, 1, None)
    assert rc == _lib.PGM_E_INVALID_ARG
    d = _lib.Dims(2, 4, 8, 17, 6, 2, 32)
    rc = L.pgm_act_forward(C.byref(d), C.c_void_p(1), C.c_void_p(1), C.c_void_p(1), 0, C.c_void_p(1),
                           C.c_void_p(1), C.c_void_p(1), None)
    assert rc == _lib.PGM_E_UNSUPPORTED and b'hidden size' in L.pgm_last_error()
    d = _lib.Dims(2, 4, 8, 19, 6, 2, 64)
    rc = L.pgm_act_forward(C.byref(d), C.c_void_p(1), C.c_void_p(1), C.c_void_p(1), 0, C.c_void_p(1),
                           C.c_void_p(1), C.c_void_p(1), None)
    assert rc == _lib.PGM_E_UNSUPPORTED and b'unsupported dims' in L.pgm_last_error()


@pytest.mark.parametrize('O,A,K', [(17, 6, 2), (11, 3, 3), (376, 17, 2)])
def test_param_layout_roundtrip(O, A, K):
    from oracle.policy import make_policy
    torch.manual_seed(3)
    pol = make_policy(O, A, K)
    sd = pol.state_dict()
    assert [k for k, _, _ in STATE_KEYS] == list(sd.keys())
    lay = ParamLayout(O, A, K)
    assert lay.total % 64 == 0
    for name, off in lay.offsets.items():
        assert off % 4 == 0
    flat = lay.flatten(sd, dtype=np.float64)
    back = lay.unflatten(flat)
    for k in sd:
        assert torch.equal(back[k], sd[k]), k
    # actor_w1 is stored transposed: element (in=k, out=j) at off + k*H + j
    w = sd['base.actor.0.weight']
    assert flat[lay.offsets['actor_w1'] + 2 * 64 + 5] == float(w[5, 2])
    n_params = sum(v.numel() for v in sd.values())
    assert n_params == 2 * (O * 64 + 64 + 64 * 64 + 64) + 64 * K + K + 64 * A + A + A


def test_adam_state_roundtrip():
    from oracle.policy import make_policy
    torch.manual_seed(0)
    pol = make_policy(17, 6, 2)
    opt = torch.optim.Adam(pol.parameters(), lr=3e-4, eps=1e-5)
    sum((q * q).sum() for q in pol.parameters()).backward()
    opt.step()
    lay = ParamLayout(17, 6, 2)
    m, v, step = lay.adam_from_optimizer_state(opt.state_dict()['state'])
    assert step == 1
    st = lay.adam_to_optimizer_state(m, v, step)
    opt2 = torch.optim.Adam(pol.parameters(), lr=3e-4, eps=1e-5)
    opt2.load_state_dict({'state': st, 'param_groups': opt.state_dict()['param_groups']})
    for i in st:
        assert torch.allclose(opt2.state_dict()['state'][i]['exp_avg'], opt.state_dict()['state'][i]['exp_avg'].float().double())


@pytest.mark.parametrize('env,P,N,T', [('MO-Walker2d-v2', 40, 4, 2048), ('MO-Hopper-v3', 27, 4, 2048),
                                       ('MO-Humanoid-v2', 20, 8, 2048), ('MO-Humanoid-v2', 3, 8, 64)])
def test_update_workspace_covers_every_split(env, P, N, T):
    """pgm_ppo_update_workspace_bytes covers the largest row split a launch may pick (PGM_NS_MAX = 4 parts per
    tower): tagged granules (the row-split updates' norm granules, 2 towers x 4 parts x 2 step parities x P + 1, then
    from granule 16 P + 8 the feature-split update's [3 kinds][P][2 towers][<= 16 parts][2 parities]; 256-B padded),
    exchange slots [P][2 towers][4 parts][2 parities], and the packed sample table + the feature-split payload
    (obs_dim <= 32: [P][2][NS][2] image slots of NB KiB and parameter slots of 4 ceil(ceil(NB / NS) / 4) KiB, NS = 16,
    the largest a launch with P' <= P tasks may pick, NB = 4 x 6 blocks for obs_dim <= 20 (compact fragments), else
    4 (ceil(O / 16) + 6)) or every workgroup's layer-1 copy
    [P][2 towers][4 parts][O H] (wide)."""
    from pgmorl_amd import envspec
    spec = envspec.make_spec(env)
    O, A, K, H = spec['obs_dim'], spec['act_dim'], spec['obj_num'], 64
    Q = max(A, K)
    d = _lib.Dims(P, N, T, O, A, K, H)
    got = _lib.lib().pgm_ppo_update_workspace_bytes(d)
    flags = -(-(16 * P + 8 + 3 * P * 2 * 16 * 2) * 8 // 256) * 256
    if O <= 32:
        img = O * H + H * (H + 1) + Q * H + 2 * H + Q + A
        xslot = -(-(img + 1) // 32) * 32
        n = O + A + 2 + 2 * K
        rs = 16 if n <= 16 else 32 if n <= 32 else 64 if n <= 64 else 128
        ns = 16
        nb = 4 * (6 if O <= 20 else -(-O // 16) + 6)
        fs = P * 2 * ns * 2 * (nb + 4 * -(-(-(-nb // ns)) // 4)) * 1024
        want = flags + P * 2 * 4 * 2 * xslot * 8 + P * T * N * rs * 4 + fs
    else:
        img = H * (H + 1) + Q * (H + 4) + 2 * H + Q + A  # head-weight rows padded to H + 4
        nkt = -(-O // 32)
        nkw = -(-nkt // 4)
        xslot = -(-((img + 4 + nkt * 32 * H + nkw * 16 * 256 + 1) // 2 + 2) // 32) * 32
        want = flags + P * 2 * 4 * 2 * xslot * 8 + P * 2 * 4 * O * H * 4  # + layer-1 copies [P][2][4][O H]
    assert got == want, (got, want)


def _fs_need(P, O):
    """Feature-split payload a launch with P tasks uses (pgm_ppo_fs.hip): NS = the largest power of two <= 16 with
    16 NS ceil(P / 8) <= 512, [P][2][NS][2] slots of NB + 4 ceil(ceil(NB / NS) / 4) KiB."""
    ns = 16
    while ns > 1 and 16 * ns * -(-P // 8) > 512:
        ns //= 2
    nb = 4 * (6 if O <= 20 else -(-O // 16) + 6)
    return P * 2 * ns * 2 * (nb + 4 * -(-(-(-nb // ns)) // 4)) * 1024 if ns >= 2 else 0


@pytest.mark.parametrize('env', ['MO-Walker2d-v2', 'MO-Hopper-v3', 'MO-Ant-v2', 'MO-Humanoid-v2'])
def test_update_workspace_is_monotone_in_tasks(env):
    """A workspace sized for a capacity of P tasks serves every launch with P' <= P active tasks (TaskBatch allocates
    once for its capacity and set_active() launches fewer): the byte count is monotone in P and covers the payload of
    the feature-split NS that P' tasks pick, which can exceed the one P tasks pick (8 parts at P' = 32, 4 at P = 33)."""
    from pgmorl_amd import envspec
    spec = envspec.make_spec(env)
    O, A, K = spec['obs_dim'], spec['act_dim'], spec['obj_num']
    L = _lib.lib()
    prev = 0
    sizes = []
    for P in range(1, 130):
        got = L.pgm_ppo_update_workspace_bytes(_lib.Dims(P, 4, 2048, O, A, K, 64))
        assert got >= prev, (P, got, prev)
        prev = got
        sizes.append(got)
    if O <= 32:
        n = O + A + 2 + 2 * K
        rs = 16 if n <= 16 else 32 if n <= 32 else 64 if n <= 64 else 128
        for cap in (33, 41, 65, 129):
            fixed = sizes[cap - 1]
            for P in range(1, cap + 1):  # the active launch's own layout: everything before the payload, then it
                flags = -(-(16 * P + 8 + 3 * P * 2 * 16 * 2) * 8 // 256) * 256
                img = O * 64 + 64 * 65 + max(A, K) * 64 + 2 * 64 + max(A, K) + A
                xslot = -(-(img + 1) // 32) * 32
                need = flags + P * 2 * 4 * 2 * xslot * 8 + P * 2048 * 4 * rs * 4 + _fs_need(P, O)
                assert need <= fixed, (cap, P, need, fixed)


@pytest.mark.parametrize('env', ['MO-Walker2d-v2', 'MO-Hopper-v2', 'MO-Hopper-v3', 'MO-Ant-v2', 'MO-Swimmer-v2'])
def test_fs_fragment_map_is_a_bijection_onto_the_tower(env):
    """pgm_ppo_fs_fragment_map (the kernels' frag_img on the host): every parameter of a tower's image -- W1 [O][H],
    W2 [H][H] of the [H][H+1] slab, the NQ head columns, b1, b2, the NQ head biases and (actor) logstd -- sits in
    exactly one (block, lane, register) slot and nothing else does; obs_dim <= 20 takes the compact layout (6 blocks
    per feature block: the head block's free columns carry the vector entries and dW1 inputs 16..19), above it
    ceil(O / 16) + 6."""
    import ctypes as C
    from pgmorl_amd import envspec
    spec = envspec.make_spec(env)
    O, A, K, H = spec['obs_dim'], spec['act_dim'], spec['obj_num'], 64
    Q = max(A, K)
    bpw = 6 if O <= 20 else -(-O // 16) + 6
    for m in (0, 1):
        NQ = K if m == 0 else A
        out = (C.c_int32 * (4 * bpw * 256))()
        nb = _lib.lib().pgm_ppo_fs_fragment_map(O, A, K, m, out, len(out))
        assert nb == 4 * bpw, (nb, bpw)
        ix = np.frombuffer(out, dtype=np.int32)
        valid = ix[ix >= 0]
        assert len(np.unique(valid)) == len(valid), 'an image entry in two slots'
        oW2 = O * H
        oWh = oW2 + H * (H + 1)
        oB1 = oWh + Q * H
        oBh = oB1 + 2 * H
        oLs = oBh + Q
        want = set(range(O * H))
        want |= {oW2 + i * (H + 1) + o for i in range(H) for o in range(H)}
        want |= {oWh + q * H + u for q in range(NQ) for u in range(H)}
        want |= set(range(oB1, oB1 + 2 * H)) | {oBh + q for q in range(NQ)}
        if m == 1:
            want |= {oLs + j for j in range(A)}
        assert set(valid.tolist()) == want, (env, m, len(valid), len(want))
    bad = (C.c_int32 * 16)()
    assert _lib.lib().pgm_ppo_fs_fragment_map(O, A, K, 0, bad, 16) < 0
    assert _lib.lib().pgm_ppo_fs_fragment_map(376, 17, 2, 0, bad, 16) < 0
