"""igr.launch - start one process per GPU for a script that was invoked as a single process.

The sharded path (igr.dist, igr.dist_train) runs as one process per GPU under
torch.distributed.  A script asked for N > 1 GPUs without a launcher around
it (`python bench.py --gpus 8`) calls `maybe_launch` first thing in main():
it starts `python -m torch.distributed.run --nproc-per-node N script args` as
a CHILD process and returns the child's exit code.  The parent never touches
the GPU: it neither initialises HIP nor replaces itself with another program
(a process that has initialised the GPU must not exec), it only waits.  The
ranks inherit stdout / stderr, so rank 0's JSON line reaches the caller as is.
"""
import os
import socket
import subprocess
import sys


def launched():
    """True inside a rank started by torch.distributed.run (or any launcher that sets
    RANK and WORLD_SIZE)."""
    return 'RANK' in os.environ and 'WORLD_SIZE' in os.environ


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def rank_command(script, argv, n_ranks, port=None):
    """The command line that runs `script argv` as n_ranks ranks on this node."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n_ranks}',
            '--master-addr', '127.0.0.1', '--master-port', str(port or free_port()),
            os.path.abspath(script)] + list(argv)


def rank_env(base=None):
    """Environment of the ranks: the caller's, with the dmabuf IPC mode RCCL needs on
    these hosts and without stale rank variables."""
    env = dict(os.environ if base is None else base)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'GROUP_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    return env


def maybe_launch(script, argv, n_ranks, one_device=False, run=subprocess.call):
    """None when this process is already a rank or n_ranks <= 1 (the caller goes on
    as rank RANK of WORLD_SIZE); otherwise starts the ranks, waits, and returns their
    exit code (non-zero if any rank failed) for the caller to exit with.

    one_device: every rank shares GPU 0 (a rehearsal on a one-GPU box), so the
    visible-device count is not checked."""
    if n_ranks <= 1 or launched():
        return None
    if not one_device:
        import torch
        have = torch.cuda.device_count()  # counts devices without initialising HIP
        if have < n_ranks:
            print(f'{os.path.basename(script)}: {n_ranks} ranks asked for but {have} GPU(s) visible '
                  f'(--one-device shares GPU 0 among the ranks for a rehearsal)', file=sys.stderr, flush=True)
            return 2
    return int(run(rank_command(script, argv, n_ranks), env=rank_env()))
