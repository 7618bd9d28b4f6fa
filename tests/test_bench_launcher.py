"""bench.py's multi-rank plumbing on CPU (gloo, --stub-cpu): `--gpus N` starts N ranks itself (the parent never
touches a GPU), torch.distributed.run with a matching --gpus works the same, a --gpus / WORLD_SIZE mismatch exits
non-zero, one failing rank ends the run non-zero, and the JSON line carries n_gpus = the ranks the collectives saw
plus the strong-scaling leg (pop 40 split in task blocks; reference fan-out morl/morl.py:84-99).
The stub replaces only the timed GPU work (a sleep per task); it is never a measurement."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, 'bench.py')


def _run(cmd, env=None, timeout=180):
    e = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e, cwd=ROOT)


def _line(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    return json.loads(lines[0])


def test_gpus2_spawns_two_ranks():
    r = _run([sys.executable, BENCH, '--gpus', '2', '--stub-cpu', '--steps', '2', '--warmup', '1'])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r)
    assert d['n_gpus'] == 2 and d['scaling'] == 'weak'
    assert d['config']['global_tasks'] == 80 and d['config']['tasks_per_gpu'] == 40
    s = d['strong']
    assert s['global_tasks'] == 40 and s['tasks_per_rank'] == [20, 20] and s['scaling'] == 'strong'
    assert d['value'] > 0 and s['value'] > 0
    assert 'STUB' in d['data']


def test_gpus3_strong_blocks():
    r = _run([sys.executable, BENCH, '--gpus', '3', '--stub-cpu', '--steps', '1', '--warmup', '0', '--tasks', '4'])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r)
    assert d['n_gpus'] == 3 and d['config']['global_tasks'] == 12
    assert d['strong']['tasks_per_rank'] == [14, 14, 12]


def test_torchrun_matching_gpus():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    r = _run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
              '--master-addr', '127.0.0.1', '--master-port', str(port), BENCH, '--gpus', '2', '--stub-cpu',
              '--steps', '1', '--warmup', '1'])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r)
    assert d['n_gpus'] == 2 and d['strong']['tasks_per_rank'] == [20, 20]


def test_gpus_world_size_mismatch_exits_nonzero():
    r = _run([sys.executable, BENCH, '--gpus', '3', '--stub-cpu'], env={'WORLD_SIZE': '2', 'RANK': '0'})
    assert r.returncode != 0 and 'WORLD_SIZE=2' in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith('{')]


def test_failing_rank_ends_the_run():
    r = _run([sys.executable, BENCH, '--gpus', '2', '--stub-cpu', '--steps', '2', '--warmup', '1'],
             env={'PGM_BENCH_STUB_FAIL_RANK': '1'})
    assert r.returncode != 0
    assert 'rank 1 exited with 3' in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith('{')]


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location('pgm_bench', BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pmc_traffic_is_quoted_only_for_the_same_variant_and_sources(tmp_path):
    """roofline.traffic comes from a PMC summary of exactly the launch the bench ran: the full
    pgm_ppo_update_variant string (family, NS, R, two per CU) and the hash of that kernel's sources.  A summary of
    another variant of the same family, or of older sources, is refused with a reason."""
    import argparse
    import json
    b = _bench_module()
    wl = 'MO-HalfCheetah-v2/P20/N4/T2048/E10/M32'
    variant = 'ppo_update_fs_kernel (NS=8, R=2, 2 per CU)'
    good = {'workload': wl, 'variant': variant, 'source_hash': b.kernel_source_hash(variant),
            'hbm_bytes_per_launch': 123.0}
    f = tmp_path / 'pmc.json'
    args = argparse.Namespace(traffic_file=str(f))
    f.write_text(json.dumps(good))
    assert b.pmc_traffic(args, wl, variant) == (123.0, str(f))
    for bad, why in ((dict(good, variant='ppo_update_fs_kernel (NS=4, R=4)'), 'not'),
                     (dict(good, source_hash='0' * 16), 'stale'),
                     (dict(good, workload='MO-HalfCheetah-v2/P10/N4/T2048/E10/M32'), 'no PMC summary')):
        f.write_text(json.dumps(bad))
        got, reason = b.pmc_traffic(args, wl, variant)
        assert got is None and why in reason, (bad, reason)
    # the committed index: every entry names its variant and source hash
    idx = json.load(open(os.path.join(ROOT, 'profiles', 'pmc_head.json')))['entries']
    for w, ent in idx.items():
        assert ent.get('variant') and ent.get('source_hash'), w
