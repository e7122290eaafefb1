"""The sharded layer's exchange pattern through RCCL (backend 'nccl') on the one GPU a
test box has: a one-rank process group.

RCCL refuses two ranks on one device, so world 1 is what can run here.  The
code path is the multi-GPU one: comm.all_reduce_sum(async_op=True) on row
slices of the item output written by the SpMMs just before it, the wait
deferred behind the NEXT layer's item-side SpMM (BipartiteShard.layer with
defer=True, as bench.py and propagate() chain layers), then the float64 MAX /
SUM reduces bench.py ends with.  At one rank the sum is the identity, so every
layer must equal the layer without the exchange bit for bit.  (A one-rank
in-place all-reduce moves no data; what this run exercises is the process
group, the stream hand-over torch wraps around every collective and the work
handles - the parts that differ from the gloo tests.)

The child process owns the process group, so nothing leaks into other tests.
"""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent('''
    import os, sys
    sys.path.insert(0, os.path.join(%(root)r, 'inductive-recommendation_amd'))
    import numpy as np, torch, torch.distributed as dist
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', device_id=dev, rank=0, world_size=1)
    from igr import comm, ops
    from igr.dist import BipartiteShard
    rng = np.random.default_rng(0)
    U, I, E, d, L = 60000, 9000, 900000, 64, 4
    u, i = rng.integers(0, U, E), rng.integers(0, I, E)
    plain = BipartiteShard.from_stream(u, i, U, I, 0, 1, dev, item_chunks=4, item_tiles=2)
    rccl = BipartiteShard.from_stream(u, i, U, I, 0, 1, dev, item_chunks=4, item_tiles=2)
    rccl.exchange = True            # issue the all-reduces although world == 1
    assert dist.get_backend() == 'nccl' and len(rccl.chunks) == 4
    g = torch.Generator(device=dev).manual_seed(1)
    xu = torch.randn(U, d, generator=g, device=dev)
    xi = torch.randn(I, d, generator=g, device=dev)
    # chained layers, every reduce deferred one layer (the pattern of bench.py / propagate)
    want_u, want_i = plain.propagate(xu, xi, L)
    got_u, got_i = rccl.propagate(xu, xi, L)
    torch.cuda.synchronize()
    assert torch.equal(got_u, want_u) and torch.equal(got_i, want_i), 'deferred exchange changed the layers'
    # one layer, waits inside the layer (dist_train's use), into caller buffers
    yu, yi = rccl.layer(xu, xi)
    wu, wi = plain.layer(xu, xi)
    torch.cuda.synchronize()
    assert torch.equal(yu, wu) and torch.equal(yi, wi)
    # the exchange explicitly, with a SpMM between issue and wait
    ref = yi.clone()
    works = [comm.all_reduce_sum(yi[r0:r1], None, async_op=True) for r0, r1, _ in rccl.chunks]
    yu2 = torch.empty_like(yu)
    ops.spmm(rccl.user_block, xi, rccl.user_vals, out=yu2)
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    assert torch.equal(yi, ref) and torch.equal(yu2, yu)
    # host-side set-up reduce and the timing reduces of bench.py
    c = comm.all_reduce_sum_host(np.arange(1000, dtype=np.int64), None, dev)
    assert np.array_equal(c, np.arange(1000))
    t = torch.tensor([1.25], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert float(t) == 1.25
    dist.barrier()
    dist.destroy_process_group()
    print('RCCL_WORLD1_OK', flush=True)
''')


def test_exchange_pattern_through_rccl_at_world_1(tmp_path):
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    script = tmp_path / 'rccl_world1.py'
    script.write_text(CHILD % {'root': ROOT})
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY='0')
    for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK'):
        env.pop(k, None)
    r = subprocess.run([sys.executable, '-u', str(script)], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0 and 'RCCL_WORLD1_OK' in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
