"""igr_spmm_noalloc_f32: the SpMM entry point that allocates nothing.

It keeps the partial rows of split rows in a static device array instead of a
caller-allocated workspace.  Called through the C ABI and compared bit for bit
with igr_spmm_f32 (whose own parity against the oracle the other GPU tests
cover) on two calls in a row, the second on a smaller graph, so stale contents
of the shared array from the first call must not leak into the second.
"""
import ctypes

import numpy as np
import pytest
import torch

from igr import _lib as L
from igr import graph as G
from oracle import igr_oracle as O

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _graph(n_rows, n_cols, nnz, seed):
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, n_rows + 1) ** 1.2
    row = rng.choice(n_rows, nnz, p=w / w.sum())
    col = rng.integers(0, n_cols, nnz)
    val = rng.standard_normal(nnz).astype(np.float32)
    g, v = G.Graph.from_coo(row, col, n_rows, n_cols, val, device=DEV, split_threshold=64, chunk_edges=64)
    assert g.n_split > 0 and g.n_chunks > g.n_split  # the chunk tier and its scratch are exercised
    return g, v


def _both(g, v, x, epi_args=None):
    """(igr_spmm_f32 with a workspace, igr_spmm_noalloc_f32) on the same inputs."""
    d = x.shape[1]
    vals = torch.from_numpy(v).to(DEV)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for name in ('igr_spmm_f32', 'igr_spmm_noalloc_f32'):
        y = torch.full((g.n_rows, d), float('nan'), device=DEV)
        args = [ctypes.byref(g.csr), d, x.data_ptr(), x.stride(0), vals.data_ptr(), y.data_ptr(), y.stride(0), None]
        if name == 'igr_spmm_f32':
            ws = torch.empty(g.n_chunks * d, device=DEV)
            args.append(ws.data_ptr())
        L.call(name, *args, st)
        torch.cuda.synchronize()
        outs.append(y)
    return outs


@pytest.mark.parametrize('d', [64, 128, 32, 256])  # every width takes the chunk tier and its scratch
def test_noalloc_matches_workspace_entry_point_twice(d):
    rng = np.random.default_rng(d)
    # first call: the larger graph; second call: a smaller one over the same array
    for n_rows, n_cols, nnz, seed in ((900, 700, 60000, 1), (300, 200, 9000, 2)):
        g, v = _graph(n_rows, n_cols, nnz, seed)
        x = torch.from_numpy(rng.standard_normal((n_cols, d)).astype(np.float32)).to(DEV)
        ref, got = _both(g, v, x)
        assert not torch.isnan(got).any()
        assert torch.equal(ref, got)
        h = g.host()
        y64 = O.spmm64(O.CSR(g.n_rows, g.n_cols, h['row_ptr'], h['col_idx'].astype(np.int64), v), x.cpu().numpy())
        err = np.abs(got.cpu().numpy() - y64)
        bound = 1e-5 * np.abs(y64) + 1e-6 * np.abs(y64).max(axis=1, keepdims=True) + 1e-30
        assert (err <= bound).all()


def test_noalloc_rejects_oversized_scratch():
    """n_chunks * d beyond the static array is an argument error, raised before any launch."""
    g, v = _graph(300, 200, 9000, 3)
    d = 64
    x = torch.zeros(200, d, device=DEV)
    y = torch.zeros(300, d, device=DEV)
    big = L.IgrCsr.from_buffer_copy(g.csr)
    big.n_chunks = L.SPMM_NOALLOC_MAX_FLOATS // d + 1
    rc = L.lib().igr_spmm_noalloc_f32(ctypes.byref(big), d, x.data_ptr(), d, None, y.data_ptr(), d, None,
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 1  # IGR_ERR_ARG
    assert b'IGR_SPMM_NOALLOC_MAX_FLOATS' in L.lib().igr_last_error()
    torch.cuda.synchronize()
    assert float(y.abs().sum()) == 0.0


def test_noalloc_under_graph_capture_replays_match():
    """The stated use: a captured hipGraph, which cannot allocate.  The first call is made
    eagerly (it looks up the array's address), the second is captured, and three replays with
    new inputs and eager work in between each equal igr_spmm_f32 bit for bit."""
    d = 64
    g, v = _graph(900, 700, 60000, 5)
    vals = torch.from_numpy(v).to(DEV)
    x = torch.randn(700, d, device=DEV)
    y = torch.full((900, d), float('nan'), device=DEV)

    def call():
        L.call('igr_spmm_noalloc_f32', ctypes.byref(g.csr), d, x.data_ptr(), x.stride(0), vals.data_ptr(),
               y.data_ptr(), y.stride(0), None, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    call()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            call()
    torch.cuda.current_stream().wait_stream(side)
    ws = torch.empty(g.n_chunks * d, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(0)
    for rep in range(3):
        x.copy_(torch.randn(700, d, device=DEV, generator=gen))
        y.fill_(float('nan'))
        graph.replay()
        torch.cuda.synchronize()
        ref = torch.empty_like(y)
        L.call('igr_spmm_f32', ctypes.byref(g.csr), d, x.data_ptr(), x.stride(0), vals.data_ptr(), ref.data_ptr(),
               ref.stride(0), None, ws.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        assert torch.equal(y, ref), f'replay {rep}'


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason='needs two GPUs')
def test_noalloc_rejects_an_output_on_another_device():
    g, v = _graph(300, 200, 9000, 3)
    d = 64
    x = torch.zeros(200, d, device='cuda:1')
    y = torch.zeros(300, d, device='cuda:1')
    with torch.cuda.device(0):
        rc = L.lib().igr_spmm_noalloc_f32(ctypes.byref(g.csr), d, x.data_ptr(), d, None, y.data_ptr(), d, None, None)
    assert rc == 1 and b'is current' in L.lib().igr_last_error()
