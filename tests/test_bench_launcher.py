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
