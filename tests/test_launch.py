"""igr.launch: a script invoked as one process starts its own ranks as children."""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from igr import graph as G
from igr import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_not_launched_when_one_rank_or_already_a_rank(monkeypatch):
    calls = []
    run = lambda cmd, env: calls.append(cmd) or 0  # noqa: E731
    monkeypatch.delenv('RANK', raising=False)
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    assert launch.maybe_launch('x.py', [], 1, run=run) is None
    monkeypatch.setenv('RANK', '0')
    monkeypatch.setenv('WORLD_SIZE', '4')
    assert launch.maybe_launch('x.py', [], 4, one_device=True, run=run) is None
    assert calls == []


def test_command_environment_and_exit_code(monkeypatch):
    monkeypatch.delenv('RANK', raising=False)
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.setenv('LOCAL_RANK', '3')  # a stale rank variable must not leak into the ranks
    monkeypatch.delenv('HSA_ENABLE_IPC_MODE_LEGACY', raising=False)
    seen = {}

    def run(cmd, env):
        seen.update(cmd=cmd, env=env)
        return 7
    rc = launch.maybe_launch('/somewhere/bench.py', ['--gpus', '4', '--steps', '2'], 4, one_device=True, run=run)
    assert rc == 7
    cmd = seen['cmd']
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node=4' in cmd and '--nnodes=1' in cmd
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[-5:] == ['/somewhere/bench.py', '--gpus', '4', '--steps', '2']
    assert seen['env']['HSA_ENABLE_IPC_MODE_LEGACY'] == '0' and 'LOCAL_RANK' not in seen['env']


def test_too_few_gpus_is_refused_without_starting_anything(monkeypatch):
    monkeypatch.delenv('RANK', raising=False)
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    import torch
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 1)
    calls = []
    assert launch.maybe_launch('x.py', [], 8, run=lambda cmd, env: calls.append(cmd) or 0) == 2
    assert calls == []


@pytest.mark.parametrize('fail_rank', [None, 1])
def test_real_ranks_see_their_environment_and_failures_propagate(tmp_path, fail_rank):
    """Two real ranks under torch.distributed.run, started by maybe_launch from a plain
    `python script.py --gpus 2`: each sees RANK / WORLD_SIZE, rank 0's line reaches stdout,
    and one failing rank makes the launcher's exit code non-zero."""
    script = tmp_path / 'ranks.py'
    script.write_text(textwrap.dedent(f'''
        import json, os, sys
        sys.path.insert(0, {os.path.join(ROOT, 'inductive-recommendation_amd')!r})
        from igr.launch import maybe_launch
        rc = maybe_launch(__file__, sys.argv[1:], 2, one_device=True)
        if rc is not None:
            sys.exit(rc)
        rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
        if rank == {fail_rank!r}:
            sys.exit(3)
        if rank == 0:
            print(json.dumps({{'n_gpus': world, 'args': sys.argv[1:], 'ipc': os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY')}}), flush=True)
    '''))
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')}
    r = subprocess.run([sys.executable, str(script), '--gpus', '2'], capture_output=True, text=True, env=env, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    if fail_rank is None:
        assert r.returncode == 0, r.stderr[-2000:]
        assert len(lines) == 1
        out = json.loads(lines[0])
        assert out == {'n_gpus': 2, 'args': ['--gpus', '2'], 'ipc': '0'}
    else:
        assert r.returncode != 0


def test_bench_starts_its_own_ranks_before_any_gpu_call():
    """`python bench.py --gpus N` on a machine without N GPUs (N = 1000: no node has that many, so
    this never starts a real run): refused by the launcher with a message (exit code 2), not an
    assertion from a rank that was never started."""
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')}
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '1000'], capture_output=True,
                       text=True, env=env, timeout=300)
    assert r.returncode == 2 and 'GPU(s) visible' in r.stderr and 'AssertionError' not in r.stderr


def test_count_ids_and_select_id_range():
    rng = np.random.default_rng(0)
    u, i = rng.integers(0, 1000, 50000), rng.integers(0, 300, 50000)
    np.testing.assert_array_equal(G.count_ids(u, 1000), np.bincount(u, minlength=1000))
    np.testing.assert_array_equal(G.count_ids(u[:0], 7), np.zeros(7, np.int64))
    for lo, hi in [(100, 400), (0, 1000), (999, 1000), (500, 500)]:
        ku, ko = G.select_id_range(u, i, lo, hi)
        m = (u >= lo) & (u < hi)
        np.testing.assert_array_equal(ku, u[m] - lo)  # stream order kept
        np.testing.assert_array_equal(ko, i[m])
    with pytest.raises(Exception, match='out of range'):
        G.count_ids(np.array([0, 5, 1000]), 1000)
