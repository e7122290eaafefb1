"""GPU parity of the HIP kernels against the CPU oracle (through the C ABI).

Tolerance (fp32): |y - y64| <= 1e-5 |y64| + 1e-6 max|y64_row|
against a float64 oracle; integer / index outputs bit-exact.
"""
import ctypes

import numpy as np
import pytest
import torch

from igr import _lib as L
from igr import graph as G
from igr import ops
from oracle import igr_oracle as O

pytestmark = pytest.mark.gpu
DEV = 'cuda'
RTOL, ATOL_ROW = 1e-5, 1e-6


def close(y, ref, rtol=RTOL, atol_row=ATOL_ROW):
    y = np.asarray(y, np.float64)
    ref = np.asarray(ref, np.float64)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    if ref.size == 0:
        return
    rowmax = np.abs(ref).max(axis=-1, keepdims=True) if ref.ndim > 1 else np.abs(ref).max()
    err = np.abs(y - ref)
    bound = rtol * np.abs(ref) + atol_row * rowmax + 1e-30
    worst = float((err / bound).max())
    assert worst <= 1.0, f'max err/bound {worst:.3g}, max abs err {err.max():.3g}'


def rand_graph(n_rows, n_cols, nnz, seed, skew=False, dedup=True, **kw):
    rng = np.random.default_rng(seed)
    if skew:
        w = 1.0 / np.arange(1, n_rows + 1) ** 1.2
        row = rng.choice(n_rows, nnz, p=w / w.sum())
    else:
        row = rng.integers(0, n_rows, nnz)
    col = rng.integers(0, n_cols, nnz)
    val = rng.standard_normal(nnz).astype(np.float32)
    g, v = G.Graph.from_coo(row, col, n_rows, n_cols, val, dedup=dedup, device=DEV, **kw)
    return g, v


def oracle_csr(g, v):
    h = g.host()
    eid = h['edge_id']
    vv = v if eid is None else v[eid]
    return O.CSR(g.n_rows, g.n_cols, h['row_ptr'], h['col_idx'].astype(np.int64), vv)


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize('d', [32, 64, 128, 256, 48, 20, 1, 300, 258])
@pytest.mark.parametrize('skew', [False, True])
def test_spmm_matches_oracle(d, skew):
    g, v = rand_graph(700, 500, 20000, seed=d, skew=skew, split_threshold=64, chunk_edges=64)
    if skew:
        assert g.n_split > 0 and g.n_chunks > g.n_split  # exercises the chunk tier + combine
    x = np.random.default_rng(9).standard_normal((500, d)).astype(np.float32)
    y = ops.spmm(g, t(x), t(v)).cpu().numpy()
    ref = O.spmm64(oracle_csr(g, v), x)
    if d == 1:  # a one-element row has no row scale to bound a cancelling sum against: the tensor's scale
        assert np.abs(y - ref).max() <= 1e-5 * np.abs(ref).max()
    else:
        close(y, ref)


def test_spmm_unit_weights_and_empty_rows():
    g, v = rand_graph(300, 100, 150, seed=5)  # most rows empty
    x = np.random.default_rng(1).standard_normal((100, 64)).astype(np.float32)
    y = ops.spmm(g, t(x)).cpu().numpy()
    A = oracle_csr(g, v)
    A.val = np.ones_like(A.val)
    close(y, O.spmm64(A, x))
    assert np.all(y[np.diff(g.host()['row_ptr']) == 0] == 0)


def test_spmm_multigraph_edge_ids():
    """DGL semantics: rhs indexed by input edge id, duplicate edges kept."""
    g, v = rand_graph(200, 150, 6000, seed=7, dedup=False, split_threshold=64, chunk_edges=64)
    assert g.edge_id is not None
    x = np.random.default_rng(2).standard_normal((150, 64)).astype(np.float32)
    y = ops.spmm(g, t(x), t(v)).cpu().numpy()
    close(y, O.spmm64(oracle_csr(g, v), x))


def test_spmm_strided_lhs_and_epilogues():
    g, v = rand_graph(400, 400, 9000, seed=11, split_threshold=64, chunk_edges=64)
    rng = np.random.default_rng(3)
    big = rng.standard_normal((400, 96)).astype(np.float32)
    x = t(big)[:, 16:80]  # leading dim 96, 16-B aligned offset
    add = rng.standard_normal((400, 64)).astype(np.float32)
    acc0 = rng.standard_normal((400, 64)).astype(np.float32)
    ref = O.spmm64(oracle_csr(g, v), np.ascontiguousarray(big[:, 16:80]))
    acc = t(acc0)
    y = ops.spmm(g, x, t(v), epi=ops.epilogue(alpha=0.5, beta=2.0, add=t(add), acc=acc, acc_mode=2, acc_div=3.0))
    yr = 0.5 * ref + 2.0 * add
    close(y.cpu().numpy(), yr, atol_row=2e-6)
    close(acc.cpu().numpy(), (acc0 + yr) / 3.0, atol_row=2e-6)
    acc2 = torch.empty_like(acc)
    ops.spmm(g, x, t(v), out=torch.empty_like(acc), epi=ops.epilogue(acc=acc2, acc_mode=1, skip_y=True))
    close(acc2.cpu().numpy(), ref)


def test_spmm_deterministic():
    g, v = rand_graph(500, 500, 40000, seed=13, skew=True, split_threshold=64, chunk_edges=64)
    x = t(np.random.default_rng(4).standard_normal((500, 64)).astype(np.float32))
    a = ops.spmm(g, x, t(v))
    for _ in range(3):
        assert torch.equal(a, ops.spmm(g, x, t(v)))


@pytest.mark.parametrize('d', [32, 64, 128])
def test_spmm_scaled_dropout_bitwise_explicit_values(d):
    """In-kernel dropout skips the gathers of dropped edges; the sums are bitwise
    those of the same SpMM with the dropped edges' values written as 0 (forward and
    reverse graph, split rows included)."""
    g, _ = rand_graph(600, 400, 30000, seed=21, skew=True, split_threshold=64, chunk_edges=64)
    assert g.n_split > 0
    rng = np.random.default_rng(d)
    rs = rng.random(600).astype(np.float32) + 0.5
    cs = rng.random(400).astype(np.float32) + 0.5
    keep, seed, off = 0.75, 5, 3
    h = g.host()
    row = np.repeat(np.arange(600), np.diff(h['row_ptr']))
    col = h['col_idx'].astype(np.int64)
    x = t(rng.standard_normal((400, d)).astype(np.float32))
    w = ops.ScaledWeights(t(rs), t(cs), keep, seed, off)
    u = ops.dropout_uniforms(g, seed, off)
    assert 0 < int((torch.floor(keep + u) == 0).sum()) < g.nnz
    vals = ops.edge_dropout(t(rs[row] * cs[col]), u, 1.0 - keep)  # forward edge ids = CSR positions
    assert torch.equal(ops.spmm_scaled(g, x, w), ops.spmm(g, x, vals))
    xr = t(rng.standard_normal((600, d)).astype(np.float32))
    rg = g.reverse()
    assert torch.equal(ops.spmm_scaled(rg, xr, w.transposed()), ops.spmm(rg, xr, vals))


@pytest.mark.parametrize('d', [32, 64, 128, 256])
def test_spmm_hub_rows_wide_combine(d):
    """Split rows averaging >= 64 chunks (the feature graph's general rows) are
    combined by 1024-thread workgroups: oracle parity, run-to-run bitwise."""
    rng = np.random.default_rng(d)
    n_rows, n_cols = 300, 4000
    row = np.concatenate([np.zeros(20000, np.int64), np.full(9000, 7), rng.integers(0, n_rows, 3000)])
    col = rng.integers(0, n_cols, len(row))
    val = rng.standard_normal(len(row)).astype(np.float32)
    g, v = G.Graph.from_coo(row, col, n_rows, n_cols, val, dedup=False, device=DEV, split_threshold=64,
                            chunk_edges=64)
    assert g.n_split >= 2 and g.n_chunks >= 64 * g.n_split
    x = rng.standard_normal((n_cols, d)).astype(np.float32)
    y = ops.spmm(g, t(x), t(v))
    close(y.cpu().numpy(), O.spmm64(oracle_csr(g, v), x))
    assert torch.equal(y, ops.spmm(g, t(x), t(v)))


def _bits_to_bool(bits, n):
    b = bits.cpu().numpy().view(np.uint32)
    return ((b[np.arange(n) >> 5] >> (np.arange(n) & 31).astype(np.uint32)) & 1).astype(bool)


def test_neighbor_and_column_masks_byte_map():
    """igr_rowset_mark_neighbors through the byte map (packed, scratch re-zeroed)
    == the set restated in numpy == the atomic-bit path; n not a multiple of 32,
    repeated rows, two calls with different rows."""
    import ctypes
    n = 1000 + 13
    g, _ = rand_graph(n, n, 30000, seed=31)
    h = g.host()
    erow = np.repeat(np.arange(n), np.diff(h['row_ptr']))
    rng = np.random.default_rng(2)
    for trial in range(2):
        rows = rng.integers(0, n, 40)
        rows[:5] = rows[5]
        for self_mark in (True, False):
            want = np.zeros(n, bool)
            want[h['col_idx'][np.isin(erow, rows)]] = True
            if self_mark:
                want[rows] = True
            got = ops.neighbor_mask(g, t(rows)) if self_mark else ops.column_mask(g, t(rows))
            np.testing.assert_array_equal(_bits_to_bool(got, n), want)
            atomic = torch.zeros((n + 31) // 32, dtype=torch.int32, device=DEV)
            ops.L.call('igr_rowset_mark_neighbors', ctypes.byref(g.csr), len(rows), ops._p(t(rows)), ops._p(atomic),
                       int(self_mark), None, ops._stream())
            assert torch.equal(atomic, got)
        assert int(ops._mark_scratch(g).sum()) == 0


def test_spmm_linearity_large():
    """Size-independent property at 1M edges: A(x1 + 2 x2) = A x1 + 2 A x2."""
    g, v = rand_graph(200000, 50000, 1000000, seed=17)
    rng = np.random.default_rng(5)
    x1 = t(rng.standard_normal((50000, 64)).astype(np.float32))
    x2 = t(rng.standard_normal((50000, 64)).astype(np.float32))
    vv = t(v)
    lhs = ops.spmm(g, x1 + 2 * x2, vv).double()
    rhs = ops.spmm(g, x1, vv).double() + 2 * ops.spmm(g, x2, vv).double()
    scale = ops.spmm(g, x1.abs() + 2 * x2.abs(), vv.abs()).double()
    assert float(((lhs - rhs).abs() - 1e-5 * scale).max()) <= 0
    # spot rows against the float64 oracle
    A = oracle_csr(g, v)
    rows = np.random.default_rng(6).choice(g.n_rows, 64, replace=False)
    y = ops.spmm(g, x1, vv).cpu().numpy()[rows]
    xs = x1.cpu().numpy()
    ref = np.stack([(A.val[A.row_ptr[r]:A.row_ptr[r + 1], None].astype(np.float64)
                     * xs[A.col[A.row_ptr[r]:A.row_ptr[r + 1]]]).sum(0) for r in rows])
    close(y, ref)


def test_sddmm_and_segment_reduce():
    g, v = rand_graph(300, 250, 6000, seed=19, dedup=False)
    rng = np.random.default_rng(7)
    for h, d in [(4, 32), (4, 64), (1, 64), (2, 24)]:
        q = rng.standard_normal((300, h * d)).astype(np.float32)
        k = rng.standard_normal((250, h * d)).astype(np.float32)
        out = ops.sddmm_dot(g, t(q), t(k), h).cpu().numpy()
        A = oracle_csr(g, v)
        ref = O.sddmm_dot(A, q.reshape(300, h, d), k.reshape(250, h, d))
        eid = g.host()['edge_id']
        # dot products cancel: bound the error by gamma_d * sum_k |q_k k_k| with gamma_d = d * 2^-24
        # (the fp32 dot-product error bound), against a float64 reference
        rows = A.rows()
        qq, kk = q.reshape(300, h, d)[rows].astype(np.float64), k.reshape(250, h, d)[A.col].astype(np.float64)
        ref64, mag = (qq * kk).sum(-1), np.abs(qq * kk).sum(-1)
        gamma = d * 2.0 ** -24
        assert np.all(np.abs(out[eid] - ref64) <= gamma * mag + 1e-30)
        assert np.all(np.abs(ref - ref64) <= gamma * mag + 1e-30)  # the oracle itself, same bound
    A = oracle_csr(g, v)
    eid = g.host()['edge_id']
    for h in [1, 2, 3, 4, 8]:  # 16-lane kernels for 1/2/4/8, the per-head kernel for 3
        x = rng.standard_normal((g.nnz, h)).astype(np.float32)
        y = ops.segment_reduce(g, t(x), 'max').cpu().numpy()
        np.testing.assert_array_equal(y, O.segment_reduce(A, x[eid], 'max'))  # max is exact
        y = ops.segment_reduce(g, t(x), 'sum').cpu().numpy()
        ref = np.zeros((g.n_rows, h))
        rows = A.rows()
        np.add.at(ref, rows, x[eid].astype(np.float64))
        mag = np.zeros((g.n_rows, h))
        np.add.at(mag, rows, np.abs(x[eid]).astype(np.float64))
        # a float sum's error is bounded by n * 2^-24 * sum |x|; rows here hold <= ~60 edges
        assert np.all(np.abs(y - ref) <= 64 * 2.0 ** -24 * mag + 1e-30)


@pytest.mark.parametrize('h,d,dedup', [(4, 64, False), (4, 64, True), (2, 128, True), (4, 32, False), (1, 64, True)])
def test_sddmm_head_split_and_long_rows(h, d, dedup):
    """Rows longer than one 64-edge block, edge-id graphs, and the head-split
    grid (one head's slice of v fits L2, the whole table does not: 6000 x 4 x 64
    floats = 6.1 MB, a slice 1.5 MB) against the float64 dot-product bound."""
    nr, nc = 400, 6000
    g, v = rand_graph(nr, nc, 60000, seed=31 + h + d, skew=True, dedup=dedup)
    rng = np.random.default_rng(8)
    q = rng.standard_normal((nr, h * d)).astype(np.float32)
    k = rng.standard_normal((nc, h * d)).astype(np.float32)
    out = ops.sddmm_dot(g, t(q), t(k), h).cpu().numpy()
    A = oracle_csr(g, v)
    eid = g.host()['edge_id']
    pos = np.arange(g.nnz) if eid is None else eid
    rows = A.rows()
    qq, kk = q.reshape(nr, h, d)[rows].astype(np.float64), k.reshape(nc, h, d)[A.col].astype(np.float64)
    ref64, mag = (qq * kk).sum(-1), np.abs(qq * kk).sum(-1)
    assert np.diff(A.row_ptr).max() > 128
    assert np.all(np.abs(out[pos] - ref64) <= d * 2.0 ** -24 * mag + 1e-30)


@pytest.mark.parametrize('h,d,dedup', [(4, 64, False), (4, 64, True), (2, 32, True), (3, 24, False)])
def test_spmm_heads_matches_per_head_oracle(h, d, dedup):
    """igr_spmm_heads_f32: head j of the output is the SpMM of x's head-j slice with
    rhs[:, j] as edge weights (by edge id), on the graph and on its reverse."""
    nr, nc = 300, 2500
    g, _ = rand_graph(nr, nc, 40000, seed=5 + h, skew=True, dedup=dedup)
    rng = np.random.default_rng(9)
    rhs = rng.standard_normal((g.nnz, h)).astype(np.float32)
    eid = g.host()['edge_id']
    for gg, n_src in [(g, nc), (g.reverse(), nr)]:
        x = rng.standard_normal((n_src, h * d)).astype(np.float32)
        y = ops.spmm_heads(gg, t(x), t(rhs), h).cpu().numpy()
        hh = gg.host()
        e2 = hh['edge_id']
        for j in range(h):
            w = np.ascontiguousarray(rhs[:, j] if e2 is None else rhs[e2, j])
            A = O.CSR(gg.n_rows, gg.n_cols, hh['row_ptr'], hh['col_idx'].astype(np.int64), w)
            ref = O.spmm64(A, x[:, j * d:(j + 1) * d])
            close(y[:, j * d:(j + 1) * d], ref)
    del eid


def test_att_softmax_forward_backward():
    g, v = rand_graph(200, 180, 4000, seed=23, skew=True)
    rng = np.random.default_rng(8)
    alpha = (rng.standard_normal((g.nnz, 4)) * 30).astype(np.float32)
    sd = ops.sqrt_scale(32)
    w = ops.att_softmax(g, t(alpha), sd)[0].cpu().numpy()
    close(w, O.att_softmax(oracle_csr(g, v), alpha, 32), rtol=2e-5)
    # backward against torch float64 autograd of the reference expression (model.py:4270-4275)
    a = t(alpha).requires_grad_(True)
    dw = t(rng.standard_normal(g.nnz).astype(np.float32))
    ops.AttSoftmax.apply(g, a, sd).backward(dw)
    a64 = torch.tensor(alpha, dtype=torch.float64, requires_grad=True)
    rows = torch.from_numpy(np.repeat(np.arange(g.n_rows), np.diff(g.host()['row_ptr'])))
    m = torch.zeros(g.n_rows, 4, dtype=torch.float64).scatter_reduce(0, rows[:, None].expand(-1, 4), a64.detach(),
                                                                     'amax', include_self=False)
    z = torch.exp((a64 - m[rows]) / sd / 10.)
    s = torch.zeros(g.n_rows, 4, dtype=torch.float64).index_add(0, rows, z)
    (z / s[rows]).mean(-1).backward(dw.cpu().double())
    close(a.grad.cpu().numpy(), a64.grad.numpy(), rtol=1e-4, atol_row=1e-5)


def test_gemm_mfma_matches_torch():
    rng = np.random.default_rng(9)
    for (m, n, k) in [(1000, 256, 64), (77, 64, 64), (130, 33, 17)]:
        a = rng.standard_normal((m, k)).astype(np.float32)
        w = rng.standard_normal((n, k)).astype(np.float32)
        b = rng.standard_normal(n).astype(np.float32)
        c = ops.gemm(t(a), t(w), t(b)).cpu().numpy()
        close(c, a.astype(np.float64) @ w.T.astype(np.float64) + b, rtol=1e-5, atol_row=1e-5)
        ct = ops.gemm(t(a.T.copy()), t(w.T.copy()), None, trans_a=True, trans_b=True).cpu().numpy()
        close(ct, a.astype(np.float64) @ w.T.astype(np.float64), rtol=1e-5, atol_row=1e-5)


def test_gather_scatter_and_bpr():
    rng = np.random.default_rng(10)
    T = rng.standard_normal((500, 64)).astype(np.float32)
    w = rng.random(64).astype(np.float32) + 0.5
    users, pos, neg = rng.integers(0, 200, 256), rng.integers(0, 300, 256), rng.integers(0, 300, 256)
    g = ops.gather_rows(t(T), t(pos), 200).cpu().numpy()
    np.testing.assert_array_equal(g, T[200 + pos])
    tt = t(T).requires_grad_(True)
    ww = t(w).requires_grad_(True)
    loss, l2 = ops.bpr_loss(tt, t(users), t(pos), t(neg), 0, 200, w=ww)
    (loss + 0.3 * l2).backward()
    T64 = torch.tensor(T, dtype=torch.float64, requires_grad=True)
    w64 = torch.tensor(w, dtype=torch.float64, requires_grad=True)
    u, p, n = T64[users], T64[200 + pos], T64[200 + neg]
    s = (u * n * w64).sum(1) - (u * p * w64).sum(1)
    rl = torch.nn.functional.softplus(s).mean()
    r2 = ((u ** 2).sum(1) + (p ** 2).sum(1) + (n ** 2).sum(1)).mean()
    (rl + 0.3 * r2).backward()
    np.testing.assert_allclose(loss.item(), rl.item(), rtol=1e-5)
    np.testing.assert_allclose(l2.item(), r2.item(), rtol=1e-5)
    close(tt.grad.cpu().numpy(), T64.grad.numpy(), rtol=1e-4, atol_row=1e-5)
    close(ww.grad.cpu().numpy(), w64.grad.numpy(), rtol=1e-4, atol_row=1e-5)


@pytest.mark.parametrize('n,arrays', [(1, 1), (5, 3), (1000, 1), (1024, 1), (1025, 2), (2048, 3), (8192, 1),
                                      (2731, 3), (70001, 1), (40000, 3)])
def test_rowsort_is_a_stable_sort_by_row(n, arrays):
    """keys = (row << 32 | entry) ascending == numpy's stable sort of the rows:
    one tile, several tiles ranked in LDS / in global memory, and > 64 tiles
    (pairwise merges first)."""
    rng = np.random.default_rng(n + arrays)
    hi = max(3, n // 7)  # many repeats
    idx = [rng.integers(0, hi, n) for _ in range(arrays)]
    offs = [0, 1000, 5][:arrays]
    args = []
    for a, o in zip(idx, offs):
        args += [t(a), o]
    keys = ops.rowsort(*args).cpu().numpy().astype(np.uint64)
    rows = np.concatenate([a + o for a, o in zip(idx, offs)]).astype(np.uint64)
    order = np.argsort(rows, kind='stable').astype(np.uint64)
    total = n * arrays
    np.testing.assert_array_equal(keys[:total], (rows[order] << np.uint64(32)) | order)


@pytest.mark.parametrize('d', [64, 128, 20])
def test_scatter_add_rows_equals_sequential_index_add_bitwise(d):
    """dst[idx[i]] += src[i] in increasing i per row: the order of a sequential
    loop over i (torch's CPU index_add_, and its index_put(accumulate=True) - the
    reference's gather backward - on one thread), hence the same bits."""
    rng = np.random.default_rng(d)
    n, rows = 6144, 900
    idx = rng.integers(0, 40, n)  # heavy repeats
    idx[n // 2:] = rng.integers(0, rows - 7, n - n // 2)
    src = rng.standard_normal((n, d)).astype(np.float32)
    dst0 = rng.standard_normal((rows, d)).astype(np.float32)
    ref = torch.from_numpy(dst0.copy())
    ref.index_add_(0, torch.from_numpy(idx + 7), torch.from_numpy(src))
    out = ops.scatter_add_rows(t(dst0.copy()), t(idx), t(src), offset=7)
    assert torch.equal(out.cpu(), ref)
    again = ops.scatter_add_rows(t(dst0.copy()), t(idx), t(src), offset=7)
    assert torch.equal(out, again)


def test_bpr_gradient_fixed_order():
    """The fused BPR gradient with repeated rows: bitwise equal run to run, equal
    to the distinct-rows form applied to gathered copies and scattered back in
    entry order, and dw bitwise equal run to run."""
    rng = np.random.default_rng(77)
    B, d = 2048, 64
    T = rng.standard_normal((600, d)).astype(np.float32)
    w = rng.random(d).astype(np.float32) + 0.5
    users, pos, neg = rng.integers(0, 150, B), rng.integers(0, 60, B), rng.integers(0, 400, B)
    runs = []
    for _ in range(2):
        tt, ww = t(T).requires_grad_(True), t(w).requires_grad_(True)
        loss, l2 = ops.bpr_loss(tt, t(users), t(pos), t(neg), 0, 200, w=ww)
        (loss + 0.3 * l2).backward()
        runs.append((tt.grad.clone(), ww.grad.clone()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])
    # the same terms through a table of gathered rows (all distinct), scattered in entry order
    rows = np.concatenate([users, 200 + pos, 200 + neg])
    gt = t(T[rows]).requires_grad_(True)
    iu, ip, ineg = ops.batch_positions(B, DEV)
    ww = t(w).requires_grad_(True)
    loss, l2 = ops.bpr_loss(gt, iu, ip, ineg, 0, 0, w=ww, distinct=True)
    (loss + 0.3 * l2).backward()
    back = ops.scatter_add_rows(torch.zeros(600, d, device=DEV), t(rows), gt.grad)
    assert torch.equal(back, runs[0][0])
    assert torch.equal(ww.grad, runs[0][1])


def test_edge_dropout_and_feat_values(golden):
    nu, ni, ta = int(golden['n_users']), int(golden['n_items']), golden['train_array']
    F = O.generate_feat(nu, ni, ta)
    g = G.Graph(F.row_ptr, F.col.astype(np.int32), F.n_rows, F.n_cols, device=DEV)
    rs = t(F.row_sum)
    for tag, alpha in [('a1', 1.0), ('a099sq', float(golden['feat_alpha_a099sq'])),
                       ('a0', float(golden['feat_alpha_a0']))]:
        fv = ops.feat_values(g, rs, (alpha - 1.) / 2. - 0.5).cpu().numpy()
        np.testing.assert_allclose(fv, golden['feat_val_' + tag], rtol=2e-7)
    rand = golden['igcn_d64_L2_train_rand']
    fv = golden['feat_val_a1']
    out = ops.edge_dropout(t(fv), t(rand), 0.3).cpu().numpy()
    ref = O.dropout_values(fv, rand, 0.3)
    np.testing.assert_array_equal(out != 0, ref != 0)  # mask bit-exact
    np.testing.assert_allclose(out, ref, rtol=1e-7)


def test_bipartite_shard_world1_matches_oracle():
    from igr.dist import BipartiteShard
    U, I, E, d = 3000, 800, 40000, 64
    rng = np.random.default_rng(12)
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)
    sh = BipartiteShard(pairs, U, I, 0, 1, DEV)
    x = rng.standard_normal((U + I, d)).astype(np.float32)
    yu, yi = sh.layer(t(x[:U]), t(x[U:]))
    y64 = O.spmm64(O.norm_adj(U, I, pairs), x)
    close(yu.cpu().numpy(), y64[:U])
    close(yi.cpu().numpy(), y64[U:])


def test_tiled_spmm_matches_oracle():
    g, v = rand_graph(3000, 20000, 120000, seed=29)
    x = np.random.default_rng(13).standard_normal((20000, 64)).astype(np.float32)
    tg = G.TiledGraph(g.host(), g.n_rows, g.n_cols, [0, 5000, 12000, 20000], DEV)
    y = ops.spmm_tiled(tg, t(x), tg.tile_values(t(v))).cpu().numpy()
    close(y, O.spmm64(oracle_csr(g, v), x), atol_row=2e-6)


def test_bipartite_shard_tiled_items():
    from igr.dist import BipartiteShard
    U, I, E, d = 20000, 500, 100000, 64
    rng = np.random.default_rng(14)
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)
    sh = BipartiteShard(pairs, U, I, 0, 1, DEV, item_tiles=3)
    assert sh.item_tiles == 3 and len(sh.chunks) == 1 and len(sh.launches()) == 4
    x = rng.standard_normal((U + I, d)).astype(np.float32)
    calls = []
    yu, yi = sh.layer(t(x[:U]), t(x[U:]), hook=lambda i, ph: calls.append((i, ph)))
    assert calls == [(i, ph) for i in range(4) for ph in ('start', 'end')]
    y64 = O.spmm64(O.norm_adj(U, I, pairs), x)
    close(yu.cpu().numpy(), y64[:U])
    close(yi.cpu().numpy(), y64[U:], atol_row=2e-6)
    # row chunks x tiles (the multi-GPU layout, run here without a process group)
    sh2 = BipartiteShard(pairs, U, I, 0, 1, DEV, item_tiles=2, item_chunks=3)
    assert len(sh2.launches()) == 7
    yu2, yi2 = sh2.layer(t(x[:U]), t(x[U:]))
    close(yi2.cpu().numpy(), y64[U:], atol_row=2e-6)
    close(yu2.cpu().numpy(), y64[:U])


def test_bipartite_shard_column_halves_at_d256(monkeypatch):
    """d = 256 with tables beyond the Infinity Cache runs both sides as two
    128-column passes (forced here on a small graph by shrinking the cache
    size): bitwise the full-width result, and both match the oracle."""
    from igr import dist as D
    U, I, E, d = 3000, 400, 40000, 256
    rng = np.random.default_rng(15)
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)
    x = rng.standard_normal((U + I, d)).astype(np.float32)
    sh = D.BipartiteShard(pairs, U, I, 0, 1, DEV, item_tiles=2, item_chunks=2)
    yu_full, yi_full = sh.layer(t(x[:U]), t(x[U:]))
    monkeypatch.setattr(D, 'MALL_BYTES', 0)
    assert D._col_width(d, 1) == 128
    yu, yi = sh.layer(t(x[:U]), t(x[U:]))
    assert torch.equal(yu, yu_full) and torch.equal(yi, yi_full)
    y64 = O.spmm64(O.norm_adj(U, I, pairs), x)
    close(yu.cpu().numpy(), y64[:U])
    close(yi.cpu().numpy(), y64[U:], atol_row=2e-6)


def test_fused_adam_matches_torch():
    from igr.optim import Adam
    rng = np.random.default_rng(15)
    p0 = rng.standard_normal(10001).astype(np.float32)
    a, b = t(p0).requires_grad_(True), t(p0).requires_grad_(True)
    oa = Adam([a], lr=1e-2, weight_decay=1e-3)
    ob = torch.optim.Adam([b], lr=1e-2, weight_decay=1e-3)
    for k in range(20):
        g = t(rng.standard_normal(10001).astype(np.float32))
        a.grad, b.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
    # same update rule; fp32 contraction differences only
    np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy(), rtol=2e-6, atol=2e-7)
    np.testing.assert_allclose(oa.state[a]['exp_avg_sq'].cpu().numpy(), ob.state[b]['exp_avg_sq'].cpu().numpy(),
                               rtol=1e-5, atol=1e-12)


def test_device_sampler_semantics():
    from igr.sampler import DeviceBPRSampler
    rng = np.random.default_rng(16)
    pairs = np.stack([rng.integers(0, 300, 5000), rng.integers(0, 120, 5000)], 1)
    pairs = pairs[pairs[:, 0] % 5 != 2]

    class DS:
        n_users, n_items, train_pairs = 300, 120, pairs

        def __len__(self):
            return len(pairs)
    s = DeviceBPRSampler(DS(), 4096, DEV, seed=3)
    u, p, n = (x.cpu().numpy() for x in s.sample(200000))
    keys = set((pairs[:, 0] * 120 + pairs[:, 1]).tolist())
    assert all(k in keys for k in (u * 120 + p).tolist())
    assert not any(k in keys for k in (u * 120 + n).tolist())
    assert np.all(u % 5 != 2)
    # users uniform over active users; negatives spread over items
    active = np.unique(pairs[:, 0])
    cnt = np.bincount(u, minlength=300)[active]
    assert cnt.min() > 0.7 * cnt.mean() and cnt.max() < 1.3 * cnt.mean()
    assert len(np.unique(n)) > 100
    # counter-based: the same (seed, offset) reproduces the batch, another offset differs
    a = s.sample(1000, offset=7)
    b = s.sample(1000, offset=7)
    c = s.sample(1000, offset=8)
    assert all(torch.equal(x, y) for x, y in zip(a, b)) and not torch.equal(a[2], c[2])


def test_device_sampler_heavy_user_gets_true_negative():
    """A user who interacted with all but two items: when the rejection rounds run
    out the negative is drawn from the complement directly, never a positive."""
    from igr.sampler import DeviceBPRSampler
    ni, free = 120, [17, 93]
    items = [i for i in range(ni) if i not in free]
    pairs = np.stack([np.zeros(len(items), np.int64), np.array(items)], 1)

    class DS:
        n_users, n_items, train_pairs = 1, ni, pairs

        def __len__(self):
            return len(pairs)
    s = DeviceBPRSampler(DS(), 4096, DEV, seed=5, max_rounds=1)
    _, _, n = (x.cpu().numpy() for x in s.sample(20000))
    assert set(np.unique(n).tolist()) == set(free)
    share = float((n == free[0]).mean())
    assert 0.45 < share < 0.55


def test_feat_values_rejects_stale_buffers():
    g, _ = rand_graph(50, 40, 300, seed=1)
    rs = torch.ones(50, device=DEV)
    with pytest.raises(ops.IgrError, match='edges'):
        ops.feat_values(g, rs, -0.5, out=torch.empty(g.nnz - 1, device=DEV))
    with pytest.raises(ops.IgrError, match='rows'):
        ops.feat_row_values(rs, -0.5, out=torch.empty(49, device=DEV))


@pytest.mark.parametrize('d', [32, 64, 128, 256])
def test_spmm_rows_and_push_match_oracle(d):
    """Row-restricted SpMM and its transpose (push), hub rows and repeated rows included."""
    n = 900
    g, v = rand_graph(n, n, 40000, seed=d + 1, skew=True)
    rng = np.random.default_rng(d)
    rows = rng.integers(0, n, 300)
    rows[:20] = 0  # the hub row, repeated
    x = rng.standard_normal((n, d)).astype(np.float32)
    ag = rng.standard_normal((n, d)).astype(np.float32)
    ai = rng.standard_normal((300, d)).astype(np.float32)
    y = ops.spmm_rows(g, t(x), t(rows), t(v), add_g=t(ag), add_i=t(ai), scale=0.25)
    full = O.spmm64(oracle_csr(g, v), x)
    close(y.cpu().numpy(), 0.25 * (full[rows] + ag[rows].astype(np.float64) + ai))
    close(ops.spmm_rows(g, t(x), t(rows)).cpu().numpy(), O.spmm64(oracle_csr(g, np.ones_like(v)), x)[rows])
    # push: dst += 0.5 * (A^T S + S), S[r] = sum of src[i] over rows[i] == r
    src = rng.standard_normal((300, d)).astype(np.float32)
    dst0 = rng.standard_normal((n, d)).astype(np.float32)
    dst = ops.spmm_push(g, t(rows), t(src), t(dst0), t(v), scale=0.5, self_add=True).cpu().numpy()
    h = g.host()
    S = np.zeros((n, d))
    np.add.at(S, rows, src.astype(np.float64))
    erow = np.repeat(np.arange(n), np.diff(h['row_ptr']))
    ref = S.copy()
    np.add.at(ref, h['col_idx'], v.astype(np.float64)[:, None] * S[erow])
    close(dst, dst0 + 0.5 * ref, atol_row=2e-6)


def test_spmm_rows_rejects_edge_id_values():
    g, v = rand_graph(50, 50, 400, seed=3, dedup=False)
    assert g.edge_id is not None
    with pytest.raises(ops.IgrError):
        ops.spmm_rows(g, t(np.zeros((50, 32), np.float32)), t(np.arange(4)), t(v))


@pytest.mark.parametrize('d', [32, 64, 128, 256])
def test_spmm_pull_marked_equals_push(d):
    """Atomic-free transpose (bitmap-masked pull) == A^T S + S, on a symmetric
    graph with a hub, repeated rows, and a second call with other rows (the
    bitmap must come back clean)."""
    n = 1000
    rng = np.random.default_rng(d + 7)
    a = rng.integers(0, n, 20000)
    b = rng.integers(0, n, 20000)
    a[:3000] = 5  # hub
    v = rng.standard_normal(20000).astype(np.float32)
    g, vv = G.Graph.from_coo(np.concatenate([a, b]), np.concatenate([b, a]), n, n, np.concatenate([v, v]),
                             dedup=True, device=DEV, symmetric=True)
    assert g.reverse() is g
    h = g.host()
    erow = np.repeat(np.arange(n), np.diff(h['row_ptr']))
    for trial in range(2):
        rows = rng.integers(0, n, 257)
        rows[:9] = 5 if trial == 0 else rows[9]
        src = rng.standard_normal((257, d)).astype(np.float32)
        y = ops.spmm_pull(g, t(rows), t(src), t(vv), scale=0.5, self_add=True).cpu().numpy()
        S = np.zeros((n, d))
        np.add.at(S, rows, src.astype(np.float64))
        ref = S.copy()
        np.add.at(ref, h['col_idx'], vv.astype(np.float64)[:, None] * S[erow])
        close(y, 0.5 * ref, atol_row=2e-6)
        push = ops.spmm_push(g, t(rows), t(src), torch.zeros(n, d, device=DEV), t(vv), scale=0.5, self_add=True)
        close(y, push.cpu().numpy().astype(np.float64), atol_row=2e-6)
        # deterministic for distinct rows (repeats are summed into their slot with float atomics)
        u = np.unique(rows)
        y1 = ops.spmm_pull(g, t(u), t(src[:len(u)]), t(vv), scale=0.5, self_add=True).cpu().numpy()
        y2 = ops.spmm_pull(g, t(u), t(src[:len(u)]), t(vv), scale=0.5, self_add=True).cpu().numpy()
        assert np.array_equal(y1, y2)
        # row_mask: the rows' neighbour set is computed bitwise as without it,
        # every other row of out is left untouched
        us = u[u != 5][:3]  # a few non-hub rows: their neighbour set leaves most rows out
        y1 = ops.spmm_pull(g, t(us), t(src[:len(us)]), t(vv), scale=0.5, self_add=True).cpu().numpy()
        nb = ops.neighbor_mask(g, t(us))
        sentinel = torch.full((n, d), 7.0, device=DEV)
        y3 = ops.spmm_pull(g, t(us), t(src[:len(us)]), t(vv), scale=0.5, self_add=True, out=sentinel,
                           row_mask=nb).cpu().numpy()
        marked = np.zeros(n, bool)
        marked[us] = True
        marked[h['col_idx'][np.isin(erow, us)]] = True
        np.testing.assert_array_equal(y3[marked], y1[marked])
        assert (y3[~marked] == 7.0).all() and (~marked).any()
    bits, filt, _ = ops._rowset(g)
    assert int(bits.abs().sum()) == 0 and int(filt.abs().sum()) == 0


@pytest.mark.parametrize('d', [64, 20])
def test_spmm_epilogue_row_scale(d):
    """y = row_scale[r] * (alpha A x + beta add), fast (d=64) and generic (d=20) kernels, split rows included."""
    g, v = rand_graph(700, 500, 20000, seed=5, skew=True, split_threshold=64, chunk_edges=64)
    rng = np.random.default_rng(1)
    x = rng.standard_normal((500, d)).astype(np.float32)
    add = rng.standard_normal((700, d)).astype(np.float32)
    rs = rng.uniform(0.1, 2.0, 700).astype(np.float32)
    y = ops.spmm(g, t(x), t(v), epi=ops.epilogue(alpha=0.5, beta=2.0, add=t(add), row_scale=t(rs)))
    ref = rs[:, None].astype(np.float64) * (0.5 * O.spmm64(oracle_csr(g, v), x) + 2.0 * add)
    close(y.cpu().numpy(), ref)


def test_spmm_pull_filter_collisions_large_graph():
    """n > 2^19: the LDS filter is not exact; columns r + 2^19 collide with marked
    rows r in the filter and must be rejected by the exact bitmap."""
    n, d = 700_000, 64
    rng = np.random.default_rng(3)
    rows = rng.integers(0, n - (1 << 19), 500)
    rows = np.concatenate([rows, rows[:50] + (1 << 19) - 1])  # some marked rows above 2^19 too
    a = np.concatenate([rng.integers(0, n, 150_000), rng.integers(0, n, 5000)])
    b = np.concatenate([rng.integers(0, n, 150_000), rows[rng.integers(0, 500, 5000)] + (1 << 19)])  # colliders
    b[-5000:] = np.minimum(b[-5000:], n - 1)
    c = np.concatenate([a[:2000], rows[:2000 % 550]])  # edges into marked rows
    a2 = np.concatenate([a, rng.integers(0, n, len(c))])
    b2 = np.concatenate([b, c])
    v = rng.standard_normal(len(a2)).astype(np.float32)
    g, vv = G.Graph.from_coo(np.concatenate([a2, b2]), np.concatenate([b2, a2]), n, n, np.concatenate([v, v]),
                             dedup=True, device=DEV, symmetric=True)
    src = rng.standard_normal((len(rows), d)).astype(np.float32)
    y = ops.spmm_pull(g, t(rows), t(src), t(vv), self_add=True).cpu().numpy()
    h = g.host()
    S = np.zeros((n, d))
    np.add.at(S, rows, src.astype(np.float64))
    erow = np.repeat(np.arange(n), np.diff(h['row_ptr']))
    ref = S.copy()
    np.add.at(ref, h['col_idx'], vv.astype(np.float64)[:, None] * S[erow])
    close(y, ref, atol_row=2e-6)
    bits, filt, _ = ops._rowset(g)
    assert int(bits.abs().sum()) == 0 and int(filt.abs().sum()) == 0


@pytest.mark.parametrize('n,m,k', [(37, 3706, 20), (5, 1_000_003, 100), (64, 130, 128), (8, 1, 1), (9, 1500, 1024)])
def test_topk_matches_sorted_reference(n, m, k):
    """igr_topk: the k largest per row, value descending, ties by index ascending
    (checked against a stable numpy sort), with many exact ties and -inf."""
    rng = np.random.default_rng(m % 1000 + k)
    s = rng.standard_normal((n, m)).astype(np.float32)
    s[:, ::7] = np.round(s[:, ::7], 1)  # exact ties
    if m > 10:
        s[0, :] = -np.inf  # a row of only -inf: the k smallest indices
        s[1, : m // 2] = 0.5  # more ties at the k-th value than needed
    val, idx = ops.topk(t(s), k)
    order = np.lexsort((np.broadcast_to(np.arange(m), s.shape), -s.astype(np.float64)), axis=1)[:, :k]
    np.testing.assert_array_equal(idx.cpu().numpy(), order)
    np.testing.assert_array_equal(val.cpu().numpy(), np.take_along_axis(s, order, 1))


@pytest.mark.parametrize('case', ['narrow', 'bin_overflow', 'unaligned', 'gowalla_row', 'k_equals_n'])
def test_topk_paths(case):
    """The two selection paths of igr_topk (candidates of the k-th value's 12-bit bin
    in LDS; radix passes over the row when that bin overflows the LDS list), float4
    and scalar row loads, against a stable numpy sort."""
    rng = np.random.default_rng(7)
    n, m, k, ld = 16, 5000, 100, None
    if case == 'narrow':  # every value in [1, 1.01): one 12-bit bin, ~1000 candidates, many ties
        s = (1 + np.round(rng.random((n, m)) * 0.01, 4)).astype(np.float32)
    elif case == 'bin_overflow':  # the k-th value's bin holds > 4096 elements
        m = 20000
        s = (1 + rng.random((n, m)) * 0.1).astype(np.float32)
        s[:, ::97] = 5.0
    elif case == 'unaligned':  # rows not 16-B aligned (odd leading dimension)
        ld = m + 3
        s = rng.standard_normal((n, m)).astype(np.float32)
    elif case == 'gowalla_row':
        n, m = 40, 40_981
        s = (rng.standard_normal((n, m)) * 0.05).astype(np.float32)
        s[:, rng.integers(0, m, 50)] = -np.inf
    else:
        m, k = 700, 700
        s = np.round(rng.standard_normal((n, m)), 1).astype(np.float32)
    if ld is None:
        x = t(s)
    else:
        buf = torch.zeros(n * ld, dtype=torch.float32, device=DEV)
        x = buf.view(n, ld)[:, 1:m + 1]  # row starts 4 B past a 16-B boundary
        x.copy_(t(s))
    val, idx = ops.topk(x, k)
    order = np.lexsort((np.broadcast_to(np.arange(m), s.shape), -s.astype(np.float64)), axis=1)[:, :k]
    np.testing.assert_array_equal(idx.cpu().numpy(), order)
    np.testing.assert_array_equal(val.cpu().numpy(), np.take_along_axis(s, order, 1))


def test_mask_scores_then_topk_matches_torch():
    """mask (absolute row_ptr slice into a bigger CSR) + topk == torch masking + sort."""
    rng = np.random.default_rng(2)
    n_all, m, k = 50, 400, 20
    lists = [sorted(set(rng.integers(0, m, rng.integers(0, 60)).tolist())) for _ in range(n_all)]
    ptr = np.concatenate([[0], np.cumsum([len(x) for x in lists])]).astype(np.int64)
    flat = np.array([i for x in lists for i in x], dtype=np.int32)
    s0, s1 = 10, 30
    sc = rng.standard_normal((s1 - s0, m)).astype(np.float32)
    gs = t(sc)
    ops.mask_scores(gs, t(ptr)[s0:s1 + 1], t(flat))
    ref = sc.copy()
    for r in range(s1 - s0):
        ref[r, lists[s0 + r]] = -np.inf
    np.testing.assert_array_equal(gs.cpu().numpy(), ref)
    _, idx = ops.topk(gs, k)
    np.testing.assert_array_equal(idx.cpu().numpy(), np.argsort(-ref, axis=1, kind='stable')[:, :k])


@pytest.mark.parametrize('m,n,k', [(256, 64, 9750), (64, 64, 20000), (130, 33, 5000), (300, 200, 1100)])
def test_gemm_split_k_matches_float64(m, n, k):
    """Few output tiles x long K (a Linear weight gradient, K = node count): K split
    over workgroups into a workspace, summed in order; every transposition and bias."""
    from igr import _lib
    assert _lib.lib().igr_gemm_workspace_size(m, n, k) > 0  # the split path is taken
    rng = np.random.default_rng(m + k)
    A = rng.standard_normal((m, k)).astype(np.float32)
    B = rng.standard_normal((k, n)).astype(np.float32)
    bias = rng.standard_normal(n).astype(np.float32)
    ref = A.astype(np.float64) @ B.astype(np.float64) + bias
    for ta in (False, True):
        for tb in (False, True):
            a = A.T.copy() if ta else A
            b = B if tb else B.T.copy()
            c = ops.gemm(t(a), t(b), t(bias), trans_a=ta, trans_b=tb).cpu().numpy()
            close(c, ref, rtol=1e-5, atol_row=1e-5)


@pytest.mark.parametrize('h', [1, 2, 3, 4, 8])
@pytest.mark.parametrize('masked', [False, True])
@pytest.mark.parametrize('multigraph', [False, True])
def test_att_softmax_heads_keep_edge_ids(h, masked, multigraph):
    """Edge softmax (model.py:4270-4275) for every head count (h = 1, 2, 4, 8: 16-lane kernels
    with register-cached rows; h = 3: the generic kernel), with dropped edges (keep == 0:
    absent from the row max / sum, weight 0) and edge-id permuted graphs; hub rows longer
    than the register cache included.  Forward and backward against float64 autograd."""
    g, _ = rand_graph(200, 180, 6000, seed=31 + h, skew=True, dedup=not multigraph)
    assert (g.edge_id is not None) == multigraph
    rng = np.random.default_rng(h + 10 * masked)
    E = g.nnz
    alpha = (rng.standard_normal((E, h)) * 30).astype(np.float32)
    keep = (rng.random(E) > 0.3).astype(np.float32) if masked else None
    sd = ops.sqrt_scale(64)
    a = t(alpha).requires_grad_(True)
    w = ops.AttSoftmax.apply(g, a, sd, None if keep is None else t(keep))
    dw = rng.standard_normal(E).astype(np.float32)
    w.backward(t(dw))
    h_ = g.host()
    rows_p = np.repeat(np.arange(g.n_rows), np.diff(h_['row_ptr']))
    rows_e = np.empty(E, np.int64)
    rows_e[h_['edge_id'] if multigraph else np.arange(E)] = rows_p
    re = torch.from_numpy(rows_e)
    a64 = torch.tensor(alpha, dtype=torch.float64, requires_grad=True)
    k = torch.ones(E, dtype=torch.bool) if keep is None else torch.from_numpy(keep != 0)
    m = torch.full((g.n_rows, h), -np.inf, dtype=torch.float64).scatter_reduce(
        0, re[k][:, None].expand(-1, h), a64.detach()[k], 'amax', include_self=True)
    z = torch.where(k[:, None], torch.exp((a64 - m[re].nan_to_num(neginf=0.)) / sd / 10.), torch.zeros(()))
    s = torch.zeros(g.n_rows, h, dtype=torch.float64).index_add(0, re, z)
    s = torch.where(s > 0, s, torch.ones(()))
    ref = torch.where(k, (z / s[re]).mean(-1), torch.zeros(()))
    ref.backward(torch.from_numpy(dw).double())
    close(w.detach().cpu().numpy(), ref.detach().numpy(), rtol=2e-5, atol_row=1e-6)
    # the gradient carries a (g - S) cancellation: bound it on the tensor's scale (h = 1 rows have one element)
    gr, g64 = a.grad.cpu().numpy().astype(np.float64), a64.grad.numpy()
    assert np.all(np.abs(gr - g64) <= 1e-4 * np.abs(g64) + 1e-5 * np.abs(g64).max())


def test_empty_graphs_and_odd_widths():
    """nnz = 0 (every row empty) and n_rows = 0 through SpMM, per-head SpMM,
    SDDMM, segment reduce and the edge softmax; d not a multiple of 4 takes the
    generic kernels."""
    g0, _ = rand_graph(5, 7, 0, seed=1)
    assert g0.nnz == 0
    x = t(np.ones((7, 64), np.float32))
    assert ops.spmm(g0, x).abs().max().item() == 0
    assert ops.spmm_heads(g0, x, torch.zeros(0, device=DEV), 2).abs().max().item() == 0
    assert ops.sddmm_dot(g0, t(np.ones((5, 64), np.float32)), x, 2).numel() == 0
    assert ops.segment_reduce(g0, torch.zeros(0, 2, device=DEV), 'max').abs().max().item() == 0
    w, _, _ = ops.att_softmax(g0, torch.zeros(0, 4, device=DEV), 8.0)
    assert w.numel() == 0
    gn, _ = rand_graph(0, 7, 0, seed=2)
    assert ops.spmm(gn, x).shape == (0, 64)
    # one value per node, the layer tail and the coefficient product on degenerate shapes
    assert ops.spmv(g0, x[:, 0].contiguous()).abs().max().item() == 0
    assert ops.spmv(gn, x[:, 0].contiguous()).shape == (0,)
    assert ops.spmm(g0, x[:, :1].contiguous()).shape == (5, 1)
    e = torch.zeros(0, 64, device=DEV)
    r0, n0 = ops.layer_tail(e, e)
    assert r0.shape == (0, 64) and n0.shape == (0, 64)
    one = t(np.array([[3.0, -4.0, 0.0]], np.float32))  # a single row, width 3: the one-float-per-lane kernel
    r1, n1 = ops.layer_tail(one, torch.zeros_like(one))
    np.testing.assert_allclose(r1.cpu().numpy(), [[3.0, -0.8, 0.0]], rtol=1e-6)
    np.testing.assert_allclose(n1.cpu().numpy(), np.array([[3.0, -0.8, 0.0]]) / np.sqrt(9.64), rtol=1e-6)
    g, v = rand_graph(60, 40, 900, seed=3)
    A = oracle_csr(g, v)
    for d in (3, 30, 66):
        xd = np.random.default_rng(d).standard_normal((40, d)).astype(np.float32)
        close(ops.spmm(g, t(xd), t(v)).cpu().numpy(), O.spmm64(A, xd))


def test_device_counters_equal_host_counters():
    """The hipGraph-step forms (a device int64 counter added on the device) give
    exactly the host-counter results: sampler batches, dropout-SpMM masks and
    Adam updates (bias corrections formed on the device)."""
    from igr import sampler as S
    from igr.optim import Adam
    rng = np.random.default_rng(4)
    pairs = np.stack([rng.integers(0, 50, 2000), rng.integers(0, 40, 2000)], 1)

    class DS:
        n_users, n_items, train_pairs = 50, 40, pairs

        def __len__(self):
            return len(pairs)
    smp = S.DeviceBPRSampler(DS(), 256, DEV, seed=9)
    ctr = torch.tensor([5], dtype=torch.int64, device=DEV)
    for a, b in zip(smp.sample(256, offset=12), smp.sample(256, offset=7, offset_dev=ctr)):
        assert torch.equal(a, b)
    g, _ = rand_graph(300, 200, 5000, seed=6)
    xs = t(rng.standard_normal((200, 64)).astype(np.float32))
    rs = t(rng.random(300).astype(np.float32))
    y1 = ops.spmm_scaled(g, xs, ops.ScaledWeights(rs, None, 0.7, 3, 12))
    y2 = ops.spmm_scaled(g, xs, ops.ScaledWeights(rs, None, 0.7, 3, 7, offset_dev=ctr))
    assert torch.equal(y1, y2)
    p1 = torch.nn.Parameter(t(rng.standard_normal(1000).astype(np.float32)))
    p2 = torch.nn.Parameter(p1.detach().clone())
    o1, o2 = Adam([p1], lr=1e-2), Adam([p2], lr=1e-2)
    steps = torch.zeros(1, dtype=torch.int64, device=DEV)
    o2.set_device_step(steps)
    for k in range(4):
        gr = t(rng.standard_normal(1000).astype(np.float32))
        p1.grad, p2.grad = gr.clone(), gr.clone()
        o1.step()
        o2.step()
        steps += 1
    torch.testing.assert_close(p2, p1, rtol=0, atol=0)


@pytest.mark.parametrize('m,n,k', [(4133, 8197, 33), (16500, 258, 70), (1000, 256, 64)])
def test_gemm_128_tiles_every_transposition(m, n, k):
    """The 128x128-tile kernel (no split and >= 2048 such tiles: the first two
    shapes; the third takes the 64-tile kernel): ragged m / n / k edges, every
    transposition, bias, against float64."""
    from igr import _lib
    assert _lib.lib().igr_gemm_workspace_size(m, n, k) == 0  # no split-K: the 128 path
    rng = np.random.default_rng(m + n + k)
    A = rng.standard_normal((m, k)).astype(np.float32)
    B = rng.standard_normal((k, n)).astype(np.float32)
    bias = rng.standard_normal(n).astype(np.float32)
    ref = A.astype(np.float64) @ B.astype(np.float64) + bias
    for ta in (False, True):
        for tb in (False, True):
            a = A.T.copy() if ta else A
            b = B if tb else B.T.copy()
            c = ops.gemm(t(a), t(b), t(bias), trans_a=ta, trans_b=tb).cpu().numpy()
            close(c, ref, rtol=1e-5, atol_row=1e-5)


@pytest.mark.parametrize('m,n,k,tb', [(4133, 256, 64, False), (1024, 64, 64, True), (33001, 256, 64, False),
                                      (40000, 128, 32, False), (70000, 512, 64, True), (20011, 64, 32, False),
                                      (17000, 128, 64, False), (1100002, 256, 64, False),
                                      (70839, 512, 128, False), (5003, 128, 128, True), (1500, 64, 128, False),
                                      (40001, 256, 128, True)])
def test_gemm_register_resident_weight_kernel(m, n, k, tb):
    """The persistent projection kernel (weight slice in registers, transposed MFMA,
    direct 16-byte C stores): short K, N in 64-column groups, M tails, every
    column-group width, bias as the accumulator's initial value, a strided A."""
    rng = np.random.default_rng(m + n + k)
    big = rng.standard_normal((m, k + 8)).astype(np.float32)
    a = t(big)[:, 4:4 + k]  # leading dimension k + 8, 16-byte aligned offset
    w = rng.standard_normal((k, n) if tb else (n, k)).astype(np.float32)
    b = rng.standard_normal(n).astype(np.float32)
    ref = big[:, 4:4 + k].astype(np.float64) @ (w if tb else w.T).astype(np.float64) + b
    c = torch.full((m, n), float('nan'), device=DEV)
    wd, bd = t(w), t(b)  # kept alive across the call
    L.call('igr_gemm_f32', m, n, k, a.data_ptr(), a.stride(0), 0, wd.data_ptr(), w.shape[1], int(tb),
           bd.data_ptr(), c.data_ptr(), n, None, 0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    close(c.cpu().numpy(), ref, rtol=1e-5, atol_row=1e-5)
    c2 = ops.gemm(t(np.ascontiguousarray(big[:, 4:4 + k])), wd, bd, trans_b=tb)
    assert torch.equal(c, c2)  # the contiguous call takes the same kernel: same bits


@pytest.mark.parametrize('h,d,dedup', [(4, 64, True), (4, 64, False), (4, 32, True), (1, 64, True), (2, 128, False),
                                       (8, 64, True), (2, 256, True), (8, 32, False), (1, 256, True)])
def test_sddmm_shared_source_and_its_gradient(h, d, dedup):
    """out[e, j] = <u[row_e, j], v[col_e]> (one source row for all heads) and
    y[r, j] = sum_e rhs[e, j] v[col_e] against float64, multigraph edge ids included,
    rows longer than a 64-edge block, empty rows; the gradient kernel is deterministic."""
    g, _ = rand_graph(300, 200, 9000, seed=h * d, skew=True, dedup=dedup)
    rng = np.random.default_rng(d + h)
    u = rng.standard_normal((300, h * d)).astype(np.float32)
    v = rng.standard_normal((200, d)).astype(np.float32)
    hst = g.host()
    row = np.repeat(np.arange(300), np.diff(hst['row_ptr']))
    col = hst['col_idx'].astype(np.int64)
    eid = hst['edge_id'] if hst['edge_id'] is not None else np.arange(g.nnz)
    out = ops.sddmm_shared(g, t(u), t(v), h).cpu().numpy()
    u64, v64 = u.astype(np.float64).reshape(300, h, d), v.astype(np.float64)
    ref = np.empty((g.nnz, h))
    ref[eid] = np.einsum('ehk,ek->eh', u64[row], v64[col])
    mag = np.empty((g.nnz, h))
    mag[eid] = np.einsum('ehk,ek->eh', np.abs(u64[row]), np.abs(v64[col]))
    assert np.all(np.abs(out - ref) <= d * 2.0 ** -24 * mag + 1e-30)
    rhs = rng.standard_normal((g.nnz, h)).astype(np.float32)
    y = ops.spmm_shared_heads(g, t(v), t(rhs), h)
    yr = np.zeros((300, h, d))
    np.add.at(yr, row, rhs.astype(np.float64)[eid][:, :, None] * v64[col][:, None, :])
    close(y.cpu().numpy(), yr.reshape(300, h * d), atol_row=2e-6)
    assert torch.equal(y, ops.spmm_shared_heads(g, t(v), t(rhs), h))
    # autograd: d/du of sum(out * rhs) is exactly that SpMM
    ut = t(u).requires_grad_(True)
    (ops.GSDDMMShared.apply(g, ut, t(v), h) * t(rhs)).sum().backward()
    assert torch.equal(ut.grad, y)


@pytest.mark.parametrize('h,d,dedup', [(4, 64, True), (1, 64, False), (2, 128, True), (8, 32, True)])
def test_sddmm_shared_source_on_a_graph_without_row_plan(h, d, dedup):
    """The same scores on a graph too large for the row plan and without split rows (more than
    2^18 rows, none above the split threshold): rows in natural order with the workgroups
    renumbered in strips per XCD (the grid is padded to whole groups of strips, so the last
    group is partly empty); runs of empty rows, rows of exactly 64 and 65 edges, rows of
    several blocks, short tails (the one-store-per-16-edges layout); multigraph edge ids."""
    n_rows, n_cols = 300_011, 5000
    rng = np.random.default_rng(h + d)
    deg = rng.integers(0, 9, n_rows)
    deg[1000:1100] = 0              # more empty rows than a wave walks
    deg[5] = 64
    deg[6] = 65
    deg[7] = 0
    deg[8] = 300
    deg[n_rows - 1] = 130
    deg[n_rows - 2] = 0
    row = np.repeat(np.arange(n_rows), deg)
    col = rng.integers(0, n_cols, len(row))
    if not dedup:  # an unsorted multigraph edge list: edge ids differ from CSR positions
        perm = rng.permutation(len(row))
        row, col = row[perm], col[perm]
    g, _ = G.Graph.from_coo(row, col, n_rows, n_cols, None, dedup=dedup, device=DEV, split_threshold=512,
                            chunk_edges=512)  # the plan of a large graph: no row of this one is split
    assert g.n_chunks == 0 and g.n_rows > (1 << 18)
    u = (rng.standard_normal((n_rows, h * d)) * 0.5).astype(np.float32)
    v = rng.standard_normal((n_cols, d)).astype(np.float32)
    out = torch.full((g.nnz, h), float('nan'), device=DEV)
    ops.sddmm_shared(g, t(u), t(v), h, out=out)
    assert not torch.isnan(out).any()
    hst = g.host()
    r_e = np.repeat(np.arange(n_rows), np.diff(hst['row_ptr']))
    c_e = hst['col_idx'].astype(np.int64)
    eid = hst['edge_id'] if hst['edge_id'] is not None else np.arange(g.nnz)
    assert dedup or hst['edge_id'] is not None
    u64, v64 = u.astype(np.float64).reshape(n_rows, h, d), v.astype(np.float64)
    ref, mag = np.empty((g.nnz, h)), np.empty((g.nnz, h))
    ref[eid] = np.einsum('ehk,ek->eh', u64[r_e], v64[c_e])
    mag[eid] = np.einsum('ehk,ek->eh', np.abs(u64[r_e]), np.abs(v64[c_e]))
    assert np.all(np.abs(out.cpu().numpy() - ref) <= d * 2.0 ** -24 * mag + 1e-30)
    assert torch.equal(out, ops.sddmm_shared(g, t(u), t(v), h))


@pytest.mark.parametrize('n', [1, 7, 1024, 2048, 5001])
def test_means_of_loss_terms(n):
    """mean(a), mean(b) in one launch: against float64, equal on repeated calls, b optional."""
    rng = np.random.default_rng(n)
    a = rng.standard_normal(n).astype(np.float32) + 0.7
    b = (rng.standard_normal(n).astype(np.float32)) ** 2
    m = ops.means(t(a), t(b))
    np.testing.assert_allclose(m.cpu().numpy(), [a.astype(np.float64).mean(), b.astype(np.float64).mean()], rtol=2e-6)
    assert torch.equal(m, ops.means(t(a), t(b)))
    m1 = ops.means(t(a))
    assert m1.shape == (1,) and torch.equal(m1[0], m[0])


def test_loss_combine_is_the_reference_expression_bitwise():
    """loss = bpr + (l2_reg * l2 + aux_reg * aux) (trainer.py:551-552) with every operation
    rounded on its own, and the running sum += loss * n, against the same tensor expression."""
    rng = np.random.default_rng(5)
    for _ in range(20):
        bpr, l2, aux = (torch.tensor(float(v), device=DEV) for v in rng.standard_normal(3).astype(np.float32))
        c_l2, c_aux, n = float(np.float32(rng.random())), float(np.float32(rng.random() * 0.1)), int(rng.integers(1, 4096))
        tot = torch.tensor(float(np.float32(rng.standard_normal())), device=DEV)
        ref = bpr + (c_l2 * l2 + c_aux * aux)
        ref_tot = tot + ref * n
        got = ops.loss_combine(bpr, l2, aux, c_l2, c_aux, loss_sum=tot, weight=n)
        assert torch.equal(got, ref) and torch.equal(tot, ref_tot)
        assert torch.equal(ops.loss_combine(bpr, l2, None, c_l2), bpr + c_l2 * l2)   # BPRTrainer, trainer.py:424-425
        assert torch.equal(ops.loss_combine(bpr), bpr)


@pytest.mark.parametrize('m,n_out,k_in', [(9748, 256, 64), (1000, 64, 64), (33001, 128, 32), (70, 64, 32), (31, 64, 64),
                                          (4133, 512, 64), (20011, 64, 32), (1100002, 256, 64),
                                          (70839, 512, 128), (5003, 128, 128), (50, 64, 128)])
def test_linear_wgrad_streamed(m, n_out, k_in):
    """dW = dy^T x and db = column sums of dy in one streamed pass (operands straight from
    global memory into the MFMAs, partial blocks of row ranges added in order): against
    float64, ranges with ragged ends, fewer rows than one group, the same bits twice, and the
    autograd path of ops.linear."""
    rng = np.random.default_rng(m + n_out + k_in)
    dy = rng.standard_normal((m, n_out)).astype(np.float32)
    x = rng.standard_normal((m, k_in)).astype(np.float32)
    dw, db = ops.linear_wgrad(t(dy), t(x))
    assert db is not None, 'the streamed kernel must take this shape'
    ref_w = dy.astype(np.float64).T @ x.astype(np.float64)
    ref_b = dy.astype(np.float64).sum(0)
    scale = np.sqrt(m)
    assert np.abs(dw.cpu().numpy() - ref_w).max() <= 2e-6 * scale * 4
    assert np.abs(db.cpu().numpy() - ref_b).max() <= 2e-6 * scale * 4
    dw2, db2 = ops.linear_wgrad(t(dy), t(x))
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    if m <= 40000:
        lin = torch.nn.Linear(k_in, n_out).to(DEV)
        xt = t(x)
        (ops.linear(xt, lin) * t(dy)).sum().backward()
        assert torch.equal(lin.weight.grad, dw) and torch.equal(lin.bias.grad, db)


def test_linear_wgrad_other_shapes_take_the_gemm():
    rng = np.random.default_rng(3)
    dy = rng.standard_normal((500, 192)).astype(np.float32)
    x = rng.standard_normal((500, 64)).astype(np.float32)
    dw, db = ops.linear_wgrad(t(dy), t(x))
    assert db is None
    close(dw.cpu().numpy(), dy.astype(np.float64).T @ x.astype(np.float64), rtol=1e-5, atol_row=1e-5)


def test_fused_adam_small_tensors_share_one_launch():
    """A model's small parameters (projection weights, biases, feature weights) go through
    igr_adam_multi_f32 in one launch: bit-identical to the per-tensor kernel, sizes that are
    not multiples of 4 or of a workgroup, more tensors than one launch holds, a device step
    counter; and the torch.optim.Adam rule to rounding."""
    from igr import optim
    rng = np.random.default_rng(21)
    sizes = [1, 3, 64, 255, 1024, 1025, 256 * 64, 70001] + [5] * 14   # 22 tensors: two launches
    init = [rng.standard_normal(n).astype(np.float32) for n in sizes]
    grads = [[rng.standard_normal(n).astype(np.float32) for n in sizes] for _ in range(4)]

    def run(small_numel, ctr=None):
        keep = optim.SMALL_NUMEL
        optim.SMALL_NUMEL = small_numel
        try:
            ps = [t(a).requires_grad_(True) for a in init]
            opt = optim.Adam(ps, lr=1e-2, weight_decay=1e-3)
            if ctr is not None:
                opt.set_device_step(ctr)
            for gs in grads:
                for p, g in zip(ps, gs):
                    p.grad = t(g)
                opt.step()
                if ctr is not None:
                    ctr.add_(1)
            return ps, opt
        finally:
            optim.SMALL_NUMEL = keep
    multi, om = run(1 << 18)
    single, os_ = run(0)
    for a, b in zip(multi, single):
        assert torch.equal(a, b)
        assert torch.equal(om.state[a]['exp_avg'], os_.state[b]['exp_avg'])
        assert torch.equal(om.state[a]['exp_avg_sq'], os_.state[b]['exp_avg_sq'])
    dev_multi, _ = run(1 << 18, torch.zeros(1, dtype=torch.int64, device=DEV))
    dev_single, _ = run(0, torch.zeros(1, dtype=torch.int64, device=DEV))
    for a, b, c in zip(dev_multi, dev_single, multi):
        assert torch.equal(a, b)
        np.testing.assert_allclose(a.detach().cpu().numpy(), c.detach().cpu().numpy(), rtol=2e-6, atol=2e-7)
    ref = [t(a).requires_grad_(True) for a in init]
    ot = torch.optim.Adam(ref, lr=1e-2, weight_decay=1e-3)
    for gs in grads:
        for p, g in zip(ref, gs):
            p.grad = t(g)
        ot.step()
    for a, b in zip(multi, ref):
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy(), rtol=2e-6, atol=2e-7)


@pytest.mark.parametrize('dedup', [True, False])
def test_edge_dropout_counter_equals_two_step_form(dedup):
    """Dropout with the uniforms drawn in the same pass == edge_dropout(val, dropout_uniforms(...)):
    the same bits, values addressed by edge id (a multigraph keeps edge ids != CSR positions),
    a device step counter, the transposed key."""
    g, _ = rand_graph(400, 300, 12000, seed=5, skew=True, dedup=dedup)
    val = torch.rand(g.nnz, device=DEV) + 0.5
    hst = g.host()
    eid = hst['edge_id']
    for swap in (False, True):
        for ctr in (None, torch.tensor([7], dtype=torch.int64, device=DEV)):
            u = ops.dropout_uniforms(g, 1234, 5, swap=swap, offset_dev=ctr)          # by CSR position
            by_eid = torch.empty_like(u)
            if eid is not None:
                by_eid[torch.from_numpy(eid.astype(np.int64)).to(DEV)] = u
            else:
                by_eid = u
            ref = ops.edge_dropout(val, by_eid, 0.3)
            got = ops.edge_dropout_counter(g, val, 0.3, 1234, 5, swap=swap, offset_dev=ctr)
            assert torch.equal(got, ref)
            assert 0.2 < float((got == 0).float().mean()) < 0.4


@pytest.mark.parametrize('dedup', [True, False])
def test_attention_kernels_split_rows_against_whole_rows(dedup):
    """The attention edge kernels take a graph's schedule: the chunks of split rows and the
    unsplit rows (SDDMM, dropout draws), chunk partials + an ordered combine (the SDDMM's
    gradient), lane groups for unsplit rows + a workgroup per split row (edge softmax and
    its backward).  Same graph under a plan that splits most rows and under one that
    splits none: per-edge results bit for bit, reductions within fp32 reassociation."""
    base, _ = rand_graph(400, 6000, 30000, seed=77, skew=True, dedup=dedup)
    hst = base.host()
    mk = lambda T, C: G.Graph(hst['row_ptr'], hst['col_idx'], 400, 6000, device=DEV, edge_id=hst['edge_id'],  # noqa: E731
                              split_threshold=T, chunk_edges=C)
    cut, whole = mk(32, 64), mk(1 << 30, 1 << 30)
    assert cut.n_split > 50 and cut.n_chunks > cut.n_split and whole.n_split == 0
    assert int(np.diff(hst['row_ptr']).max()) > 2048  # a hub row longer than a workgroup's register cache
    h, d = 4, 64
    rng = np.random.default_rng(5)
    u = t(rng.standard_normal((400, h * d)).astype(np.float32))
    v = t(rng.standard_normal((6000, d)).astype(np.float32))
    rhs = t(rng.standard_normal((base.nnz, h)).astype(np.float32))
    assert torch.equal(ops.sddmm_shared(cut, u, v, h), ops.sddmm_shared(whole, u, v, h))
    assert torch.equal(ops.sddmm_shared(cut, u[:, :d].contiguous(), v, 1), ops.sddmm_shared(whole, u[:, :d].contiguous(), v, 1))
    y_cut, y_whole = ops.spmm_shared_heads(cut, v, rhs, h), ops.spmm_shared_heads(whole, v, rhs, h)
    close(y_cut.cpu().numpy(), y_whole.cpu().numpy(), rtol=1e-5, atol_row=2e-6)
    assert torch.equal(y_cut, ops.spmm_shared_heads(cut, v, rhs, h))  # ordered combine: same bits again
    val = t(rng.standard_normal(base.nnz).astype(np.float32))
    for swap in (False, True):
        assert torch.equal(ops.edge_dropout_counter(cut, val, 0.3, 99, 3, swap=swap),
                           ops.edge_dropout_counter(whole, val, 0.3, 99, 3, swap=swap))
    sd = ops.sqrt_scale(d)
    keep = t((rng.random(base.nnz) > 0.3).astype(np.float32))
    dw = t(rng.standard_normal(base.nnz).astype(np.float32))
    for kp in (None, keep):
        res = []
        for g in (cut, whole):
            a = (rhs * 30).clone().requires_grad_(True)
            g.max_row_edges = 1 << 30  # the chunked path whatever the row lengths (the default takes it above 8192 edges)
            w = ops.AttSoftmax.apply(g, a, sd, kp)
            w.backward(dw)
            res.append((w.detach().cpu().numpy(), a.grad.cpu().numpy()))
        close(res[0][0], res[1][0], rtol=2e-5, atol_row=1e-6)
        gr, g0 = res[0][1].astype(np.float64), res[1][1].astype(np.float64)
        assert np.all(np.abs(gr - g0) <= 1e-4 * np.abs(g0) + 1e-5 * np.abs(g0).max())
        # the plain entry points (no workspace): a workgroup per split row
        import ctypes
        from igr import _lib as L
        a = (rhs * 30).contiguous()
        P = lambda x: None if x is None else ctypes.c_void_p(x.data_ptr())  # noqa: E731
        w2, rmax, rsum = torch.empty(base.nnz, device=DEV), torch.empty(400, h, device=DEV), torch.empty(400, h, device=DEV)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.call('igr_att_softmax_f32', ctypes.byref(cut.csr), h, P(a), P(kp), float(sd), P(w2), P(rmax), P(rsum), st)
        close(w2.cpu().numpy(), res[1][0], rtol=2e-5, atol_row=1e-6)
        da = torch.empty_like(a)
        L.call('igr_att_softmax_bwd_f32', ctypes.byref(cut.csr), h, P(a), P(kp), float(sd), P(rmax), P(rsum), P(dw), P(da), st)
        gr = da.cpu().numpy().astype(np.float64)
        assert np.all(np.abs(gr - g0) <= 1e-4 * np.abs(g0) + 1e-5 * np.abs(g0).max())


@pytest.mark.parametrize('seed', range(16))
def test_random_shapes_and_schedules_match_oracle(seed):
    """Shapes, degree distributions, duplicate edges, widths and row schedules drawn at random
    (the automatic schedule included): SpMM both ways, the shared-head SDDMM and the edge
    softmax against the oracle on the same inputs."""
    rng = np.random.default_rng(1000 + seed)
    n_rows, n_cols = int(rng.integers(1, 4000)), int(rng.integers(1, 4000))
    nnz = int(rng.integers(0, 150000))
    skew, dedup = bool(rng.integers(2)), bool(rng.integers(2))
    plan = {} if rng.integers(3) == 0 else dict(split_threshold=int(rng.choice([16, 48, 64, 256, 512, 1 << 30])),
                                                chunk_edges=int(rng.choice([64, 128, 192, 512, 4096])))
    d = int(rng.choice([32, 64, 128, 256, int(rng.integers(1, 300))]))
    print(f'seed {seed}: {n_rows} x {n_cols}, nnz {nnz}, skew {skew}, dedup {dedup}, plan {plan}, d {d}', flush=True)
    g, v = rand_graph(n_rows, n_cols, nnz, seed=seed, skew=skew, dedup=dedup, **plan)
    A = oracle_csr(g, v)
    x = rng.standard_normal((n_cols, d)).astype(np.float32)
    y = ops.spmm(g, t(x), t(v)).cpu().numpy()
    ref = O.spmm64(A, x)
    bound = 1e-5 * np.abs(ref) + 2e-6 * max(np.abs(ref).max(initial=0.), 1e-30)  # tensor scale: d may be 1
    assert np.all(np.abs(y - ref) <= bound)
    # one value per node (the width-1 product)
    yv = ops.spmv(g, t(np.ascontiguousarray(x[:, 0])), t(v)).cpu().numpy()
    ref1 = O.spmm64(A, np.ascontiguousarray(x[:, :1]))[:, 0]
    mag = O.spmm64(O.CSR(n_rows, n_cols, A.row_ptr, A.col, np.abs(A.val)), np.abs(x[:, :1]))[:, 0]
    assert np.all(np.abs(yv - ref1) <= 2e-6 * mag + 1e-30)
    # the transposed product, as the backward takes it: the reverse graph reads values by edge id
    r = g.reverse()
    gy = rng.standard_normal((n_rows, d)).astype(np.float32)
    gx = ops.spmm(r, t(gy), t(v)).cpu().numpy()
    hr = r.host()
    At = O.CSR(n_cols, n_rows, hr['row_ptr'], hr['col_idx'].astype(np.int64), v[hr['edge_id']])
    ref = O.spmm64(At, gy)
    bound = 1e-5 * np.abs(ref) + 2e-6 * max(np.abs(ref).max(initial=0.), 1e-30)
    assert np.all(np.abs(gx - ref) <= bound)
    if g.nnz == 0:
        return
    # attention edge kernels (widths the shared-head kernels are built for)
    h, da = (4, 64) if seed % 2 else (1, 32)
    q = rng.standard_normal((n_rows, h * da)).astype(np.float32)
    k = rng.standard_normal((n_cols, da)).astype(np.float32)
    s = ops.sddmm_shared(g, t(q), t(k), h).cpu().numpy().reshape(g.nnz, h)
    rows = A.rows()
    qq = q.reshape(n_rows, h, da)[rows].astype(np.float64)
    kk = k[A.col].astype(np.float64)[:, None, :]
    s64, mag = (qq * kk).sum(-1), np.abs(qq * kk).sum(-1)
    eid = g.host()['edge_id']
    s_csr = s if eid is None else s[eid]  # per-edge outputs are in edge-id order
    assert np.all(np.abs(s_csr - s64) <= da * 2.0 ** -23 * mag + 1e-30)
    alpha = (rng.standard_normal((g.nnz, h)) * 30).astype(np.float32)
    w = ops.att_softmax(g, t(alpha), ops.sqrt_scale(da))[0].cpu().numpy()
    a_csr = alpha if eid is None else alpha[eid]
    w_ref = O.att_softmax(A, a_csr, da)
    close(w if eid is None else w[eid], w_ref, rtol=2e-5)
    rhs = rng.standard_normal((g.nnz, h)).astype(np.float32)
    yh = ops.spmm_shared_heads(g, t(k), t(rhs), h).cpu().numpy()
    r_csr = rhs if eid is None else rhs[eid]
    for j in range(h):
        ref = O.spmm64(O.CSR(n_rows, n_cols, A.row_ptr, A.col, np.ascontiguousarray(r_csr[:, j])), k)
        close(yh[:, j * da:(j + 1) * da], ref, atol_row=2e-6)


@pytest.mark.parametrize('d', [32, 64, 100, 128, 256])
@pytest.mark.parametrize('drop', [False, True])
def test_layer_tail_matches_torch(d, drop):
    """r = dropout(leaky_relu(a + b, 0.2)), nrm = F.normalize(r) (model.py:4040-4042) in one
    kernel each way against the torch float64 expression with the same mask: both outputs,
    the gradient from both outputs (the normalised one arriving as a column block of a wider
    gradient), from one of them alone, and an all-zero row (the norm's clamp)."""
    n = 1003
    rng = np.random.default_rng(d)
    a = rng.standard_normal((n, d)).astype(np.float32)
    b = rng.standard_normal((n, d)).astype(np.float32)
    a[7], b[7] = 0., 0.
    keep = (rng.random((n, d)) > 0.3).astype(np.float32) if drop else None
    scale = 1 / 0.7 if drop else 1.0
    wide = rng.standard_normal((n, 3 * d)).astype(np.float32)
    gr = rng.standard_normal((n, d)).astype(np.float32)

    def ref(use_r, use_n):
        a64 = torch.tensor(a, dtype=torch.float64, requires_grad=True)
        b64 = torch.tensor(b, dtype=torch.float64, requires_grad=True)
        r = torch.nn.functional.leaky_relu(a64 + b64, 0.2)
        if drop:
            r = r * torch.tensor(keep, dtype=torch.float64) * scale
        nrm = torch.nn.functional.normalize(r, p=2, dim=1)
        loss = 0.
        if use_r:
            loss = loss + (r * torch.tensor(gr, dtype=torch.float64)).sum()
        if use_n:
            loss = loss + (nrm * torch.tensor(wide[:, d:2 * d], dtype=torch.float64)).sum()
        loss.backward()
        return r.detach().numpy(), nrm.detach().numpy(), a64.grad.numpy(), b64.grad.numpy()

    for use_r, use_n in [(True, True), (False, True), (True, False)]:
        at, bt = t(a).requires_grad_(True), t(b).requires_grad_(True)
        r, nrm = ops.LayerTail.apply(at, bt, None if keep is None else t(keep), scale, 0.2)
        loss = 0.
        if use_r:
            loss = loss + (r * t(gr)).sum()
        if use_n:
            loss = loss + (torch.cat([r.detach(), nrm, r.detach()], 1) * t(wide)).sum()
        loss.backward()
        r64, n64, ga, gb = ref(use_r, use_n)
        close(r.detach().cpu().numpy(), r64, rtol=1e-6)
        close(nrm.detach().cpu().numpy(), n64, rtol=2e-6, atol_row=1e-7)
        close(at.grad.cpu().numpy(), ga, rtol=2e-5, atol_row=2e-6)
        assert torch.equal(at.grad, bt.grad)
    assert np.all(nrm.detach().cpu().numpy()[7] == 0)


def test_gspmm_backward_streams_permuted_values():
    """gspmm's backward permutes the edge values into the reverse graph's order once per value
    tensor and streams them (Graph.positional): the same bits as reading them through the
    edge ids - over two chained layers sharing the tensor, again after an in-place change of
    the values, and for another value tensor."""
    g, v = rand_graph(400, 400, 20000, seed=3, skew=True)
    rev = g.reverse()
    assert rev.edge_id is not None and rev.positional().edge_id is None
    rng = np.random.default_rng(3)
    dy = t(rng.standard_normal((400, 64)).astype(np.float32))

    def check(values):
        x = t(rng.standard_normal((400, 64)).astype(np.float32)).requires_grad_(True)
        y2 = ops.gspmm(g, 'mul', 'sum', ops.gspmm(g, 'mul', 'sum', x, values), values)
        (y2 * dy).sum().backward()
        assert torch.equal(x.grad, ops.spmm(rev, ops.spmm(rev, dy, values), values))

    vals = t(v)
    check(vals)
    check(vals)
    vals.mul_(2.0)
    check(vals)
    check(t(rng.standard_normal(g.nnz).astype(np.float32)))


@pytest.mark.parametrize('n,k,d', [(9746, 2, 64), (9746, 1, 64), (70001, 3, 128), (5, 2, 32)])
def test_coef_product_and_its_gradient(n, k, d):
    """out = coef @ b with gradient-free per-row coefficients (IMCGAE's repeated blocks): the
    product and d b = coef^T g (the split-K GEMM over all rows, g a column block of a wider
    gradient) against float64; the same bits twice."""
    rng = np.random.default_rng(n + k)
    coef = rng.standard_normal((n, k)).astype(np.float32)
    b = rng.standard_normal((k, d)).astype(np.float32)
    wide = rng.standard_normal((n, 2 * d)).astype(np.float32)
    grads = []
    for _ in range(2):
        bt = t(b).requires_grad_(True)
        out = ops.coef_product(t(coef), bt)
        (torch.cat([out, out.detach()], 1) * t(wide)).sum().backward()
        grads.append(bt.grad)
    close(out.detach().cpu().numpy(), coef.astype(np.float64) @ b.astype(np.float64), atol_row=2e-6)
    ref = coef.astype(np.float64).T @ wide[:, :d].astype(np.float64)
    assert np.abs(grads[0].cpu().numpy() - ref).max() <= 4e-6 * np.sqrt(n) * 4
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize('dedup', [True, False])
def test_spmv_matches_oracle(dedup):
    """y[r] = sum_p rhs[eid(p)] x[col[p]] (one value per node): hub rows through the schedule's
    split list, unsplit and empty rows, duplicate edges read by edge id, unit weights, a graph
    without a schedule; the same bits twice."""
    for kw in (dict(split_threshold=32, chunk_edges=64), dict(split_threshold=1 << 30, chunk_edges=64), {}):
        g, v = rand_graph(900, 5000, 40000, seed=41, skew=True, dedup=dedup, **kw)
        if kw.get('split_threshold') == 32:
            assert g.n_split > 20 and g.n_order + g.n_split == g.n_rows
        x = np.random.default_rng(2).standard_normal(5000).astype(np.float32)
        A = oracle_csr(g, v)
        mag = O.spmm64(O.CSR(900, 5000, A.row_ptr, A.col, np.abs(A.val)), np.abs(x)[:, None])[:, 0]
        y = ops.spmv(g, t(x), t(v))
        assert np.all(np.abs(y.cpu().numpy() - O.spmm64(A, x[:, None])[:, 0]) <= 2e-6 * mag + 1e-30)
        assert torch.equal(y, ops.spmv(g, t(x), t(v)))
        A.val = np.ones_like(A.val)
        y1 = ops.spmv(g, t(x)).cpu().numpy()
        mag1 = O.spmm64(A, np.abs(x)[:, None])[:, 0]
        assert np.all(np.abs(y1 - O.spmm64(A, x[:, None])[:, 0]) <= 2e-6 * mag1 + 1e-30)
        empty = np.diff(g.host()['row_ptr']) == 0
        assert empty.any() and np.all(y1[empty] == 0)


def test_gspmm_backward_permuted_copy_lives_with_its_values():
    """The reverse-order copy of the edge values is dropped when the value tensor dies and kept
    while it lives (a model's persistent values: one permutation for the whole training)."""
    import gc
    g, v = rand_graph(300, 300, 8000, seed=9, skew=True)
    rev = g.reverse()
    dy = t(np.random.default_rng(1).standard_normal((300, 32)).astype(np.float32))

    def run(values):
        x = t(np.random.default_rng(2).standard_normal((300, 32)).astype(np.float32)).requires_grad_(True)
        (ops.gspmm(g, 'mul', 'sum', x, values) * dy).sum().backward()
        return x.grad

    keep = t(v)
    g1 = run(keep)
    held = rev.__dict__['_perm_cache'][2]
    assert torch.equal(run(keep), g1) and rev.__dict__['_perm_cache'][2] is held  # reused, not redone
    run(t(v) * 2)  # a temporary value tensor ...
    gc.collect()
    assert '_perm_cache' not in rev.__dict__  # ... takes its copy with it
