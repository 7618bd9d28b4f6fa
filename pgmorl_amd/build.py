"""Build libpgm.so (gfx950) with hipcc and libpgm_host.so with g++, in-tree.  ``python -m pgmorl_amd.build``."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, 'libpgm.so')
OBJDIR = os.path.join(HERE, 'build')
SOURCES = ['pgm_abi.cpp', 'pgm_policy_env.hip', 'pgm_rollout_lanes.hip', 'pgm_rollout_wide.hip', 'pgm_misc.hip', 'pgm_ppo_update.hip',
           'pgm_ppo_mfma.hip', 'pgm_ppo_fs.hip', 'pgm_ppo_wide.hip']
HEADERS = ['pgm_common.hpp', 'pgm_dispatch.hpp', 'pgm_rollout.hpp', 'pgm_mfma.hpp', 'pgm_ppo_shared.hpp']
ARCH = os.environ.get('PGM_OFFLOAD_ARCH', 'gfx950')
FLAGS = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-I', os.path.join(ROOT, 'include')]


def _hipcc():
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', 'hipcc'):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return 'hipcc'


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths)


HOST_LIB = os.path.join(HERE, 'libpgm_host.so')


def build_host(force=False, verbose=False):
    """libpgm_host.so: the native generation-boundary path (include/pgm_host.h), host C++ only (g++)."""
    src = os.path.join(CSRC, 'pgm_host.cpp')
    hdr = os.path.join(ROOT, 'include', 'pgm_host.h')
    if not force and os.path.exists(HOST_LIB) and os.path.getmtime(HOST_LIB) >= _newest([src, hdr]):
        return HOST_LIB
    cmd = [os.environ.get('CXX', 'g++'), '-O2', '-std=c++17', '-fPIC', '-shared', '-pthread', '-I',
           os.path.join(ROOT, 'include'), src, '-o', HOST_LIB]
    if verbose:
        print(' '.join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'g++ failed on pgm_host.cpp:\n{r.stdout}\n{r.stderr}')
    return HOST_LIB


TEST_LIB = os.path.join(HERE, 'libpgm_test.so')


def build(force=False, verbose=False, stamps=False, test_hooks=False):
    """stamps=True builds the diagnostic libpgm_stamps.so (-DPGM_STAMPS phase timers); never shipped.
    test_hooks=True builds libpgm_test.so: the production objects with pgm_abi.cpp recompiled -DPGM_TEST_HOOKS (the
    PGM_TEST_DELAY exchange stall and the PGM_TEST_RESIDENT_CUS co-residency override, read by the test build only;
    tests/test_gpu_exchange.py loads it through _lib.test_build())."""
    if test_hooks:
        return _build_test(force=force, verbose=verbose)
    objdir = OBJDIR + ('_stamps' if stamps else '')
    lib = LIB.replace('libpgm.so', 'libpgm_stamps.so') if stamps else LIB
    flags = FLAGS + (['-DPGM_STAMPS'] if stamps else [])
    os.makedirs(objdir, exist_ok=True)
    deps = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, 'include', 'pgm_abi.h')]
    dep_t = _newest(deps)
    hipcc = _hipcc()

    def compile_one(src):
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, src + '.o')
        if not force and os.path.exists(o) and os.path.getmtime(o) >= max(os.path.getmtime(s), dep_t):
            return o
        cmd = [hipcc, *flags, '-c', s, '-o', o]
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed on {src}:\n{r.stdout}\n{r.stderr}')
        return o

    if not stamps:
        build_host(force=force, verbose=verbose)
    with ThreadPoolExecutor(max_workers=min(4, len(SOURCES))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    if force or not os.path.exists(lib) or os.path.getmtime(lib) < _newest(objs):
        cmd = [hipcc, f'--offload-arch={ARCH}', '-shared', '-fPIC', *objs, '-o', lib]
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc link failed:\n{r.stdout}\n{r.stderr}')
    return lib


def _build_test(force=False, verbose=False):
    build(force=force, verbose=verbose)
    hipcc = _hipcc()
    objdir = OBJDIR + '_test'
    os.makedirs(objdir, exist_ok=True)
    src = os.path.join(CSRC, 'pgm_abi.cpp')
    o = os.path.join(objdir, 'pgm_abi.cpp.o')
    deps = [src] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, 'include', 'pgm_abi.h')]
    if force or not os.path.exists(o) or os.path.getmtime(o) < _newest(deps):
        cmd = [hipcc, *FLAGS, '-DPGM_TEST_HOOKS', '-c', src, '-o', o]
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed on pgm_abi.cpp (test hooks):\n{r.stdout}\n{r.stderr}')
    objs = [o] + [os.path.join(OBJDIR, s + '.o') for s in SOURCES if s != 'pgm_abi.cpp']
    if force or not os.path.exists(TEST_LIB) or os.path.getmtime(TEST_LIB) < _newest(objs):
        cmd = [hipcc, f'--offload-arch={ARCH}', '-shared', '-fPIC', *objs, '-o', TEST_LIB]
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc link failed (test build):\n{r.stdout}\n{r.stderr}')
    return TEST_LIB


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True, stamps='--stamps' in sys.argv,
                test_hooks='--test' in sys.argv))
