"""GPU parity at the size of BASELINE's configurations (not only toy graphs).

    MovieLens-1M shape, d = 64, 2 layers, attention SpMM   AttIGCN  model.py:4223-4287
    Gowalla shape (29,858 x 40,981, ~1.04 M), d = 128, L = 3  IGCN     model.py:4188-4200, config.py:12-23
    synthetic scale, d = 256, the sharded layer with 128-column passes
    the bench workload itself (10 M x 1 M, 200 M draws, d = 64) through size-independent properties
    the same graph at d = 256 (BASELINE's 8-GPU configuration's layer, here on one GPU), likewise
    the attention edge kernels on that graph's feature graph (nnz 411 M, 4 heads of d = 64), likewise
    items outnumbering users (Amazon-Books-shaped: 2.9 M items x 600 K users, d = 128), items cut
    into ranges: at world 1 through the properties, at world 2 on one GPU against world 1; and a
    tenth of that shape at world 2 against the float64 oracle

The first two compare against fixtures written by tests/golden/make_scale_golden.py,
which RAN the reference on the same inputs (data from tests/golden/ml_like.py,
parameters from numpy streams; the fixtures keep float64 column sums and sampled
rows), and against the CPU oracle.  Tolerances as in test_gpu_models: 1e-5
relative + 1e-6 of the row max for SpMM-type outputs (3e-5 / 3e-6 through the
attention softmax), 1e-4 / 1e-5 for gradients through it; index arrays exact.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN
from igr import model as M
from oracle import igr_oracle as O
from test_gpu_kernels import close

sys.path.insert(0, GOLDEN)
import ml_like  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda')


class DS:
    def __init__(self, name, n_users, n_items, train):
        self.name, self.n_users, self.n_items = name, n_users, n_items
        self.train_data = train
        lens = np.array([len(x) for x in train], np.int64)
        flat = np.fromiter((i for x in train for i in x), np.int64, count=int(lens.sum()))
        self.train_pairs = np.stack([np.repeat(np.arange(n_users, dtype=np.int64), lens), flat], 1)
        self.train_array = self.train_pairs

    def __len__(self):
        return len(self.train_pairs)


def _load(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.skip(f'{path} not generated')
    return np.load(path)


def check_summary(fx, key, t, rows, rtol=1e-5, atol_row=1e-6, sum_tol=2e-6):
    """Sampled rows against the reference's, and the float64 column sums of the
    whole tensor within sum_tol of its sum of magnitudes."""
    a = t.detach().cpu().numpy()
    close(a[rows], fx[key + '_rows'], rtol=rtol, atol_row=atol_row)
    cs = a.astype(np.float64).sum(0)
    assert np.abs(cs - fx[key + '_colsum']).max() <= sum_tol * float(fx[key + '_abssum']), key
    assert float(np.abs(a.astype(np.float64)).sum()) == pytest.approx(float(fx[key + '_abssum']), rel=1e-5)


def test_attigcn_at_ml1m_shape_matches_reference():
    """BASELINE configuration 2: attention SpMM at the MovieLens-1M shape, d = 64, L = 2."""
    fx = _load('scale_att_ml1m.npz')
    nu, ni, _, d, L, _ = ml_like.SHAPES['ml1m']
    train, _, _ = ml_like.splits_for('ml1m')
    ds = DS('ml1m', nu, ni, train)
    assert len(ds) == int(fx['n_train'])
    cfg = {'name': 'AttIGCN', 'embedding_size': d, 'n_layers': L, 'device': DEV, 'dropout': 0.3,
           'feature_ratio': 1., 'dataset': ds, 'dropout_rng': 'cpu'}
    m = M.AttIGCN(cfg)
    assert m.feat_mat.nnz == int(fx['nnz_feat'])
    P = ml_like.scale_params('att_ml1m', m.embedding.weight.shape[0], d, heads=4)
    S = ml_like.scale_samples('att_ml1m', nu + ni, m.feat_mat.nnz)
    with torch.no_grad():
        m.embedding.weight.copy_(torch.from_numpy(P['emb']))
        for lin, w, b in [(m.weight_q, 'wq', 'bq'), (m.weight_k, 'wk', 'bk')]:
            lin.weight.copy_(torch.from_numpy(P[w]))
            lin.bias.copy_(torch.from_numpy(P[b]))
    m.eval()
    with torch.no_grad():
        alpha = m.inductive_rep_layer(m.feat_vals, return_alpha=True)
        close(alpha.cpu().numpy()[S['edges']], fx['alpha_edges'], rtol=3e-5, atol_row=2e-6)
        assert float(alpha.double().sum()) == pytest.approx(float(fx['alpha_sum']), rel=1e-6)
        x0 = m.inductive_rep_layer(m.feat_vals)
        check_summary(fx, 'x0', x0, S['rows'], rtol=3e-5, atol_row=3e-6)
    # the CPU oracle's restatement of the same layer (model.py:4257-4281) on the full graph
    F = O.generate_feat(nu, ni, ds.train_pairs)
    fv = O.feat_values(F, 0.0)
    np.testing.assert_array_equal(m.feat_mat.host()['col_idx'], F.col.astype(np.int32))
    x0_o, w_o = O.att_x0(F, fv, P['emb'], P['wq'], P['bq'], P['wk'], P['bk'])
    close(alpha.cpu().numpy(), w_o, rtol=3e-5, atol_row=2e-6)
    close(x0.cpu().numpy(), x0_o, rtol=3e-5, atol_row=3e-6)
    rep = m.get_rep()
    check_summary(fx, 'rep', rep, S['rows'], rtol=3e-5, atol_row=3e-6)
    R = torch.from_numpy(ml_like.scale_cotangent(tuple(rep.shape))).to(DEV)
    (rep * R).sum().backward()
    check_summary(fx, 'grad_emb', m.embedding.weight.grad, S['feat_rows'], rtol=1e-4, atol_row=1e-5, sum_tol=1e-5)
    for g, k in [(m.weight_q.weight.grad, 'grad_wq'), (m.weight_k.weight.grad, 'grad_wk')]:
        ref = fx[k].astype(np.float64)
        assert np.abs(g.cpu().numpy() - ref).max() <= 1e-4 * np.abs(ref).max(), k
    assert np.abs(m.weight_q.bias.grad.cpu().numpy() - fx['grad_bq']).max() <= 1e-4 * np.abs(fx['grad_bq']).max()
    # train mode: the reference's own dropout draws (CPU generator); dropped edges leave the softmax
    m.train()
    torch.manual_seed(33)
    with torch.no_grad():
        check_summary(fx, 'train_rep', m.get_rep(), S['rows'], rtol=3e-5, atol_row=3e-6)


def test_igcn_at_gowalla_shape_matches_reference():
    """BASELINE configuration 3: IGCN at the Gowalla shape, d = 128, L = 3 (config.py:12-23)."""
    fx = _load('scale_igcn_gowalla.npz')
    nu, ni, _, d, L, _ = ml_like.SHAPES['gowalla']
    train, _, _ = ml_like.splits_for('gowalla')
    ds = DS('gowalla', nu, ni, train)
    assert len(ds) == int(fx['n_train'])
    m = M.IGCN({'name': 'IGCN', 'embedding_size': d, 'n_layers': L, 'device': DEV, 'dropout': 0.3,
                'feature_ratio': 1., 'dataset': ds, 'dropout_rng': 'cpu'})
    assert m.feat_mat.nnz == int(fx['nnz_feat']) and m.norm_adj.nnz == int(fx['nnz_adj'])
    P = ml_like.scale_params('igcn_gowalla', m.embedding.weight.shape[0], d)
    S = ml_like.scale_samples('igcn_gowalla', nu + ni, m.feat_mat.nnz, m.norm_adj.nnz)
    # degree / normalisation work: bit-exact against the reference's values
    np.testing.assert_array_equal(m.norm_vals.cpu().numpy()[S['adj_edges']], fx['norm_val_edges'])
    assert float(m.norm_vals.double().sum()) == float(fx['norm_val_sum'])
    with torch.no_grad():
        m.embedding.weight.copy_(torch.from_numpy(P['emb']))
    m.eval()
    rep = m.get_rep()
    check_summary(fx, 'rep', rep, S['rows'])
    # float64 oracle on the whole graph
    A, F = O.norm_adj(nu, ni, ds.train_pairs), O.generate_feat(nu, ni, ds.train_pairs)
    x = O.spmm64(F, P['emb'], val=O.feat_values(F, 1.0))
    acc = x.copy()
    for _ in range(L):
        x = _spmm64_f64(A, x)
        acc += x
    close(rep.detach().cpu().numpy(), acc / (L + 1), rtol=1e-5, atol_row=2e-6)
    (rep * torch.from_numpy(ml_like.scale_cotangent(tuple(rep.shape))).to(DEV)).sum().backward()
    check_summary(fx, 'grad_emb', m.embedding.weight.grad, S['feat_rows'], rtol=2e-5, atol_row=2e-6, sum_tol=1e-5)
    m.train()
    torch.manual_seed(31)
    with torch.no_grad():
        check_summary(fx, 'train_rep', m.get_rep(), S['rows'])


def _spmm64_f64(A, x64):
    """A x with float64 input (scipy): the layers of the float64 reference chain."""
    import scipy.sparse as sp
    mat = sp.csr_matrix((A.val.astype(np.float64), A.col, A.row_ptr), shape=(A.n_rows, A.n_cols))
    return mat @ x64


def test_sharded_layer_d256_column_passes_at_scale():
    """BASELINE configuration 5's layer (d = 256) on one GPU at a size where the item
    table (300 K x 1 KB = 307 MB) outgrows the Infinity Cache, so both sides run as two
    128-column passes: float64 spot rows, linearity of the whole layer, and bitwise
    equality with the single-pass path."""
    from igr import dist
    from igr.dataset import synthetic_pairs
    U, I, E, d = 1_000_000, 300_000, 20_000_000, 256
    pairs = synthetic_pairs(U, I, E, 5, 'uniform')
    sh = dist.BipartiteShard(pairs, U, I, 0, 1, DEV, d=d, item_tiles=2)
    assert dist._col_width(d, I * d * 4) == 128
    g = torch.Generator(device=DEV).manual_seed(1)
    xu, xi = torch.randn(U, d, generator=g, device=DEV) * 0.1, torch.randn(I, d, generator=g, device=DEV) * 0.1
    yu, yi = sh.layer(xu, xi)
    # float64 on sampled rows of both sides
    rng = np.random.default_rng(0)
    ub, ih = sh.user_block.host(), sh.item_host
    xi_h, xu_h = xi.cpu().numpy().astype(np.float64), xu.cpu().numpy().astype(np.float64)
    uv, iv = sh.user_vals.cpu().numpy().astype(np.float64), ih['vals'].astype(np.float64)
    for r in rng.integers(0, U, 64):
        b, e = ub['row_ptr'][r], ub['row_ptr'][r + 1]
        close(yu[r].cpu().numpy()[None], (uv[b:e, None] * xi_h[ub['col_idx'][b:e]]).sum(0)[None])
    for r in rng.integers(0, I, 64):
        b, e = ih['row_ptr'][r], ih['row_ptr'][r + 1]
        close(yi[r].cpu().numpy()[None], (iv[b:e, None] * xu_h[ih['col_idx'][b:e]]).sum(0)[None], atol_row=2e-6)
    # linearity: layer(a x + b z) == a layer(x) + b layer(z) to rounding
    zu, zi = torch.randn(U, d, generator=g, device=DEV) * 0.1, torch.randn(I, d, generator=g, device=DEV) * 0.1
    wu, wi = sh.layer(zu, zi)
    cu, ci = sh.layer(0.5 * xu - 2.0 * zu, 0.5 * xi - 2.0 * zi)
    for got, a, b in [(cu, yu, wu), (ci, yi, wi)]:
        ref = 0.5 * a.double() - 2.0 * b.double()
        scale = float(ref.abs().max())
        assert float((got.double() - ref).abs().max()) <= 2e-6 * scale
    # the column passes change no bit
    one = dist._col_width
    try:
        dist._col_width = lambda d_, table_bytes: d_
        vu, vi = sh.layer(xu, xi)
    finally:
        dist._col_width = one
    assert torch.equal(vu, yu) and torch.equal(vi, yi)


def _layer_properties(sh, d, seed=2, n_sample=200, single_pass_equal=False):
    """One propagation layer of a world-1 shard, checked through properties that need no second
    full-size implementation.  `cut` is the side the shard cuts into ranges (rows of
    user_block), `rep` the replicated side:
      * a known answer: sqrt(degree) is an eigenvector of D^-1/2 A D^-1/2 with eigenvalue 1
        (utils.py:42-50), so layer(sqrt(deg)) = sqrt(deg) on every node with an interaction;
      * float64 on sampled rows of both sides, from the host CSR;
      * the adjoint identity <x_c, A_cr x_r> = <A_rc x_c, x_r> ties the two blocks together;
      * column checksums: 1^T (A x) = (A^T 1)^T x with the column sums of A taken on the host;
      * linearity, and the same bits on a second run;
      * single_pass_equal: the 128-column passes of a wide layer change no bit."""
    from igr import dist
    C, R = sh.u1 - sh.u0, sh.n_items
    deg = torch.from_numpy(sh.degree).to(DEV)
    # known answer (fp32 values: three roundings per edge, ~20 to ~200 terms per row)
    sc, sr = deg[:C].sqrt()[:, None].repeat(1, d).contiguous(), deg[C:].sqrt()[:, None].repeat(1, d).contiguous()
    ec, er = sh.layer(sc, sr)
    for got, ref in [(ec, sc), (er, sr)]:
        assert float(((got - ref).abs() / ref.clamp_min(1.0)).max()) <= 1e-5
    del sc, sr, ec, er
    g = torch.Generator(device=DEV).manual_seed(seed)
    xc, xr = torch.randn(C, d, generator=g, device=DEV) * 0.1, torch.randn(R, d, generator=g, device=DEV) * 0.1
    yc, yr = sh.layer(xc, xr)
    # sampled rows in float64
    rng = np.random.default_rng(0)
    ub, ih = sh.user_block.host(), sh.item_host
    uv, iv = sh.user_vals.cpu().numpy(), ih['vals']
    for r in rng.integers(0, C, n_sample):
        b, e = int(ub['row_ptr'][r]), int(ub['row_ptr'][r + 1])
        src = xr[torch.from_numpy(ub['col_idx'][b:e].astype(np.int64)).to(DEV)].cpu().numpy().astype(np.float64)
        close(yc[r].cpu().numpy()[None], (uv[b:e, None].astype(np.float64) * src).sum(0)[None], atol_row=2e-6)
    heavy = np.argsort(np.diff(ih['row_ptr']))[-8:]  # the longest rows of the replicated side (split-row path)
    for r in np.concatenate([rng.integers(0, R, n_sample), heavy]):
        b, e = int(ih['row_ptr'][r]), int(ih['row_ptr'][r + 1])
        src = xc[torch.from_numpy(ih['col_idx'][b:e].astype(np.int64)).to(DEV)].cpu().numpy().astype(np.float64)
        close(yr[r].cpu().numpy()[None], (iv[b:e, None].astype(np.float64) * src).sum(0)[None], atol_row=2e-6)
    # adjoint identity between the two blocks (A symmetric)
    lhs = float((xc.double() * yc.double()).sum())   # <x_c, A_cr x_r>
    rhs = float((yr.double() * xr.double()).sum())   # <A_rc x_c, x_r>
    scale = float((xc.double().abs() * yc.double().abs()).sum())
    assert abs(lhs - rhs) <= 1e-6 * scale
    # column checksums against host column sums of the values (float64)
    cs_rep = np.bincount(ub['col_idx'], weights=uv.astype(np.float64), minlength=R)   # A_cr^T 1
    cs_cut = np.bincount(ih['col_idx'], weights=iv.astype(np.float64), minlength=C)   # A_rc^T 1
    for y, cs, x in [(yc, cs_rep, xr), (yr, cs_cut, xc)]:
        got = y.double().sum(0).cpu().numpy()
        w = torch.from_numpy(cs).to(DEV)
        ref = (w[:, None] * x.double()).sum(0).cpu().numpy()
        mag = float((w[:, None] * x.double().abs()).sum(0).max())
        assert np.abs(got - ref).max() <= 1e-6 * mag
    del cs_rep, cs_cut
    # linearity and repeatability
    zc, zr = torch.randn(C, d, generator=g, device=DEV) * 0.1, torch.randn(R, d, generator=g, device=DEV) * 0.1
    wc, wr = sh.layer(zc, zr)
    cc, cr = sh.layer(0.5 * xc - 2.0 * zc, 0.5 * xr - 2.0 * zr)
    for got, a, b in [(cc, yc, wc), (cr, yr, wr)]:
        ref = 0.5 * a.double() - 2.0 * b.double()
        assert float((got.double() - ref).abs().max()) <= 2e-6 * float(ref.abs().max())
        del ref
    del zc, zr, wc, wr, cc, cr
    vc, vr = sh.layer(xc, xr)
    assert torch.equal(vc, yc) and torch.equal(vr, yr)
    if single_pass_equal:
        one = dist._col_width
        try:
            dist._col_width = lambda d_, table_bytes: d_
            vc, vr = sh.layer(xc, xr)
        finally:
            dist._col_width = one
        assert torch.equal(vc, yc) and torch.equal(vr, yr)
    return xc, xr, yc, yr


_STREAM = {}


def _bench_stream():
    """The bench workload's pair stream (10 M users x 1 M items, 200 M draws, seed 0), drawn once."""
    from igr.dataset import synthetic_pairs
    if 'ui' not in _STREAM:
        _STREAM['ui'] = synthetic_pairs(10_000_000, 1_000_000, 200_000_000, 0, 'uniform', stacked=False)
    return _STREAM['ui']


def test_bench_workload_full_size_properties():
    """The bench workload itself (10 M users x 1 M items, 200 M draws, d = 64: the graph, the
    values and the launches bench.py times; one layer is model.py:4193-4197) - see
    _layer_properties."""
    from igr import dist
    U, I, d = 10_000_000, 1_000_000, 64
    u, i = _bench_stream()
    sh = dist.BipartiteShard.from_stream(u, i, U, I, 0, 1, DEV, d=d)
    assert sh.local_nnz == 399_995_952 and sh.item_tiles == 4  # the graph and the tiling of the bench line
    _layer_properties(sh, d)


def test_bench_graph_partition_for_8_ranks_full_size():
    """The 8-GPU configuration's partition at its size (host side only: the shards are built on
    the CPU, one rank after the other, with the degree all-reduce replaced by the other ranks'
    counts): eight contiguous user ranges that cover every user, ~50 M edges each (both
    directions), the same four item row chunks on every rank, all 399,995,952 edges owned once."""
    from igr import dist
    from igr.graph import count_ids
    U, I, W = 10_000_000, 1_000_000, 8
    u, i = _bench_stream()
    E = len(u)
    total = np.concatenate([count_ids(u, U), count_ids(i, I)])
    nnz, prev, cuts = [], 0, None
    for r in range(W):
        e0, e1 = E * r // W, E * (r + 1) // W
        others = total - np.concatenate([count_ids(u[e0:e1], U), count_ids(i[e0:e1], I)])
        sh = dist.BipartiteShard.from_stream(u, i, U, I, r, W, 'cpu', reduce=lambda c, o=others: c + o)
        assert sh.u0 == prev and sh.item_tiles == 1 and sh.user_block.nnz == sh.item_nnz
        prev = sh.u1
        c = [(a, b) for a, b, _ in sh.chunks]
        assert len(c) == 4 and (cuts is None or c == cuts)
        cuts = c
        nnz.append(sh.local_nnz)
        del sh
    assert prev == U and sum(nnz) == 399_995_952
    assert max(nnz) - min(nnz) < 1000, nnz  # balanced to within a few users' edges


def test_synthetic_d256_full_size_properties():
    """BASELINE configuration 5's layer at its full size: the same 10 M x 1 M x 200 M-draw graph
    at d = 256 (one layer of model.py:4193-4197), which runs as two 128-column passes over
    8 source tiles on the item side and over the 1 GB item table on the user side.  The
    property set of _layer_properties, plus: the column passes change no bit against the
    single-pass path, over the whole output."""
    from igr import dist
    U, I, d = 10_000_000, 1_000_000, 256
    u, i = _bench_stream()
    sh = dist.BipartiteShard.from_stream(u, i, U, I, 0, 1, DEV, d=d)
    assert sh.local_nnz == 399_995_952 and sh.item_tiles == 8
    assert dist._col_width(d, I * d * 4) == 128
    _layer_properties(sh, d, seed=4, n_sample=100, single_pass_equal=True)
    _STREAM.clear()


def test_amazon_books_shape_full_size_properties():
    """BASELINE configuration 4's graph at its size on one GPU: items outnumber users
    (2.9 M items x 600 K users, 30 M draws with Zipf item popularity, d = 128; the layout the
    Amazon loader produces, dataset.py:229-255), so the ITEMS are the side cut into ranges
    and the user block is the replicated, all-reduced one (sharded_side).  World 1 here; the
    world-2 run of the same graph is test_items_sharded_world2_full_size."""
    from igr import dist
    sh = _amazon_shard(0, 1, DEV)
    assert sh.n_items == AM_U and sh.u1 - sh.u0 == AM_I  # the shard's cut side is the items
    _layer_properties(sh, AM_D, seed=6)


def test_attention_kernels_full_size_properties():
    """The attention inductive layer's edge kernels on IGCN's feature graph of the synthetic
    bipartite graph (11 M nodes, nnz 411 M, 4 heads of d = 64; model.py:4246-4275):
      * shared-source SDDMM on sampled edges against float64;
      * the adjoint identity sum_{r,h} <u[r,h], y[r,h]> = sum_{e,h} rhs[e,h] out[e,h] between
        the SDDMM (out) and its gradient kernel (y = sum_e rhs[e,h] v[col_e]);
      * the edge softmax: weights in [0, 1], each row's weights sum to 1, sampled rows against
        a float64 softmax of the scores (mean over heads, model.py:4270-4275);
      * the segmented max equals the max over each sampled row's scores; same bits twice."""
    from igr import ops
    from igr.dataset import synthetic_pairs
    from igr.dist_train import FeatureShard
    U, I, E, d, H = 10_000_000, 1_000_000, 200_000_000, 64, 4
    pairs = synthetic_pairs(U, I, E, 0)
    g = FeatureShard(pairs, U, I, 0, U, 0, DEV).graph
    del pairs
    assert g.nnz == 410_995_952
    gen = torch.Generator(device=DEV).manual_seed(3)
    u = torch.randn(g.n_rows, H * d, device=DEV, generator=gen) * 0.1
    v = torch.randn(g.n_cols, d, device=DEV, generator=gen) * 0.1
    out = ops.sddmm_shared(g, u, v, H)
    assert torch.equal(out, ops.sddmm_shared(g, u, v, H))
    hst = g.host()
    rp, ci = hst['row_ptr'], hst['col_idx']
    eid = hst['edge_id']
    rng = np.random.default_rng(1)
    rows = rng.integers(0, g.n_rows, 300)
    for r in rows:
        b, e = int(rp[r]), int(rp[r + 1])
        if b == e:
            continue
        ids = torch.from_numpy((eid[b:e] if eid is not None else np.arange(b, e)).astype(np.int64)).to(DEV)
        vc = v[torch.from_numpy(ci[b:e].astype(np.int64)).to(DEV)].double()       # [deg, d]
        ref = torch.einsum('hd,ed->eh', u[r].double().view(H, d), vc)               # [deg, H]
        got = out[ids].double()
        assert float((got - ref).abs().max()) <= 1e-5 * float(ref.abs().max()) + 1e-7
        # the segmented max over this row's scores
    smax = ops.segment_reduce(g, out, 'max')
    for r in rows[:100]:
        b, e = int(rp[r]), int(rp[r + 1])
        if b == e:
            continue
        ids = torch.from_numpy((eid[b:e] if eid is not None else np.arange(b, e)).astype(np.int64)).to(DEV)
        assert torch.equal(smax[r], out[ids].max(0).values)
    # adjoint identity with the gradient kernel
    rhs = torch.randn(g.nnz, H, device=DEV, generator=gen)
    y = ops.spmm_shared_heads(g, v, rhs, H)
    lhs = float((u.double() * y.double()).sum())
    rsum_ = float((rhs.double() * out.double()).sum())
    scale = float((rhs.double().abs() * out.double().abs()).sum())
    assert abs(lhs - rsum_) <= 1e-6 * scale
    del rhs, y
    # edge softmax (mean over heads of the per-head row softmax of out / sqrt(d) / 10)
    w, rmax, rsum = ops.att_softmax(g, out, ops.sqrt_scale(d))
    assert float(w.min()) >= 0.0 and float(w.max()) <= 1.0 + 1e-6
    tot = ops.segment_reduce(g, w, 'sum')
    deg = torch.from_numpy(np.diff(rp)).to(DEV)
    assert float((tot[deg > 0] - 1.0).abs().max()) <= 1e-5
    for r in rows[:100]:
        b, e = int(rp[r]), int(rp[r + 1])
        if b == e:
            continue
        ids = torch.from_numpy((eid[b:e] if eid is not None else np.arange(b, e)).astype(np.int64)).to(DEV)
        ref = torch.softmax(out[ids].double() / float(np.float32(np.sqrt(d))) / 10., 0).mean(1)
        assert float((w[ids].double() - ref).abs().max()) <= 3e-6


@pytest.mark.parametrize('mode', ['eval', 'train'])
def test_igcn_forward_backward_adjoint_at_training_scale(mode):
    """IGCN's get_rep is linear in the embedding table (model.py:4188-4200: rep = P E, P the
    layer mean of powers of A applied to the inductive layer F), so its backward must be the
    transpose: <G, P E> = <P^T G, E>.  On a 1 M x 100 K x 20 M-draw graph (d = 64, L = 3), in
    eval mode and in train mode, where the forward and the reverse feature SpMM have to draw
    the same in-kernel dropout mask (model.py:4189, 4019-4028) for the identity to hold.
    Also: the row-restricted path (last layer only at a batch's rows) equals those rows of
    the full rep."""
    from igr import ops
    from igr.dataset import synthetic_pairs
    U, I, E, d = 1_000_000, 100_000, 20_000_000, 64
    pairs = synthetic_pairs(U, I, E, 0)

    class Data:
        name = 'synthetic'
        n_users, n_items, train_pairs = U, I, pairs
        train_array = pairs
        train_data = None

        def __len__(self):
            return len(pairs)
    torch.manual_seed(0)
    m = M.IGCN({'name': 'IGCN', 'embedding_size': d, 'n_layers': 3, 'device': DEV, 'dropout': 0.3,
                'feature_ratio': 1., 'dataset': Data(), 'batch_rep': False})
    m.train(mode == 'train')
    gen = torch.Generator(device=DEV).manual_seed(7)
    G = torch.randn(U + I, d, device=DEV, generator=gen)
    rep = m.get_rep()
    (rep * G).sum().backward()
    emb = m.embedding.weight
    lhs = float((G.double() * rep.detach().double()).sum())
    rhs = float((emb.grad.double() * emb.detach().double()).sum())
    scale = float((G.double().abs() * rep.detach().double().abs()).sum())
    assert abs(lhs - rhs) <= 2e-6 * scale, (lhs, rhs, scale)
    if mode == 'eval':
        with torch.no_grad():
            rows = torch.randint(0, U + I, (6144,), device=DEV, generator=gen)
            rb = ops.propagate_rows(m.norm_adj, emb, m.n_layers, rows, feat=m.feat_mat, fvals=m.inductive_values(),
                                    adj_vals=m.norm_vals)
            ref = rep.detach()[rows]
            assert float((rb - ref).abs().max()) <= 1e-5 * float(ref.abs().max())


# ---------------------------------------------------------------- items outnumber users, items sharded (world 2)

AM_U, AM_I, AM_E, AM_D = 600_000, 2_900_000, 30_000_000, 128


def _amazon_shard(rank, world, dev, group=None):
    """Shard `rank` of the Amazon-Books-shaped graph, items cut into ranges."""
    from igr.dataset import synthetic_pairs
    from igr.dist import BipartiteShard, sharded_side
    assert sharded_side(AM_U, AM_I, 'auto') == 'items'
    u, i = synthetic_pairs(AM_U, AM_I, AM_E, 9, 'zipf', stacked=False)
    return BipartiteShard.from_stream(i, u, AM_I, AM_U, rank, world, dev, group=group, d=AM_D)


def _am_inputs(dev):
    g = torch.Generator(device=dev).manual_seed(12)
    return (torch.randn(AM_I, AM_D, generator=g, device=dev) * 0.1,
            torch.randn(AM_U, AM_D, generator=g, device=dev) * 0.1)


def _am_step(n_rows):
    """Row sampling stride: ~3000 rows of a rank's range (Zipf popularity gives the first
    rank a few hundred very long rows, the last one millions of short ones)."""
    return max(1, n_rows // 3000)


def _am_full_rank(rank, world, port, q):
    import torch.distributed as tdist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        dev = torch.device('cuda')
        sh = _amazon_shard(rank, world, dev)
        x_items, x_users = _am_inputs(dev)
        y_own, y_rep = sh.layer(x_items[sh.u0:sh.u1].contiguous(), x_users)
        y2_own, y2_rep = sh.propagate(x_items[sh.u0:sh.u1].contiguous(), x_users, 2)
        torch.cuda.synchronize()
        # hand back samples and checksums, not 1.8 GB of rows
        rows_own = torch.arange(0, sh.u1 - sh.u0, _am_step(sh.u1 - sh.u0), device=dev)
        q.put((rank, sh.u0, sh.u1, sh.local_nnz, y_own[rows_own].cpu().numpy(), y_rep.cpu().numpy(),
               y2_own[rows_own].cpu().numpy(), y2_rep.cpu().numpy(),
               y_own.double().sum(0).cpu().numpy(), y2_own.double().sum(0).cpu().numpy()))
    except Exception:
        import traceback
        q.put((rank, 'error', traceback.format_exc()))
    finally:
        tdist.destroy_process_group()


def test_items_sharded_world2_full_size():
    """BASELINE configuration 4 at its size as TWO ranks (both on the one GPU; gloo, staged
    through host memory): rank-local set-up from the shared stream, one layer and two chained
    layers with deferred reduces, against the world-1 shard of the same graph on this GPU:
    the replicated user block must agree to fp32 reassociation of the two partial sums, the
    unsplit item rows of each rank bit for bit (they are complete locally once x is the same)."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_am_full_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
    for r in res:
        assert r[1] != 'error', r[2]
    one = _amazon_shard(0, 1, DEV)
    x_items, x_users = _am_inputs(DEV)
    y_items, y_users = one.layer(x_items, x_users)
    y2_items, y2_users = one.propagate(x_items, x_users, 2)
    assert res[0][1] == 0 and res[-1][2] == AM_I and res[0][2] == res[1][1]
    assert sum(r[3] for r in res) == one.local_nnz
    tot1, tot2, n_short, n_split = np.zeros(AM_D), np.zeros(AM_D), 0, 0
    deg_items = np.diff(one.user_block.host()['row_ptr'])
    for rank, i0, i1, _nnz, y_own, y_rep, y2_own, y2_rep, s1, s2 in res:
        rows = torch.arange(0, i1 - i0, _am_step(i1 - i0), device=DEV) + i0
        # layer 1: an item row needs only x_users, so a rank's rows equal the world-1 rows bit
        # for bit - except rows long enough to be split into chunks (> 512 edges), whose
        # partial sums are added in a tree chosen from the shard's chunk statistics
        want = y_items[rows].cpu().numpy()
        short = deg_items[rows.cpu().numpy()] <= 512
        n_short, n_split = n_short + int(short.sum()), n_split + int((~short).sum())
        assert np.array_equal(y_own[short], want[short]), 'unsplit item rows differ between world 2 and world 1'
        close(y_own, want, atol_row=2e-6)
        close(y_rep, y_users.cpu().numpy(), atol_row=2e-6)
        close(y2_own, y2_items[rows].cpu().numpy(), rtol=2e-5, atol_row=3e-6)
        close(y2_rep, y2_users.cpu().numpy(), rtol=2e-5, atol_row=3e-6)
        tot1 += s1
        tot2 += s2
    assert n_short > 1000 and n_split >= 1  # both kinds of row were compared
    np.testing.assert_allclose(tot1, y_items.double().sum(0).cpu().numpy(), rtol=1e-6, atol=1e-5)  # split rows differ in the last bit
    np.testing.assert_allclose(tot2, y2_items.double().sum(0).cpu().numpy(), rtol=1e-5, atol=1e-6)
    # both ranks hold the same reduced user block, bit for bit
    assert np.array_equal(res[0][5], res[1][5]) and np.array_equal(res[0][7], res[1][7])


AMS_U, AMS_I, AMS_E = 52_000, 290_000, 3_000_000  # a tenth of the shape, against the float64 oracle


def _amazon_pairs():
    from igr.dataset import synthetic_pairs
    return synthetic_pairs(AMS_U, AMS_I, AMS_E, 9, 'zipf')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _am_rank(rank, world, port, q):
    import torch.distributed as tdist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from igr.dist import BipartiteShard, sharded_side
        dev = torch.device('cuda')
        pairs = _amazon_pairs()
        side = sharded_side(AMS_U, AMS_I, 'auto')
        assert side == 'items'
        sw = np.ascontiguousarray(pairs[:, ::-1])  # the shard cuts its first side: items
        sh = BipartiteShard(sw, AMS_I, AMS_U, rank, world, dev, d=AM_D)
        rng = np.random.default_rng(3)
        x_items = (rng.standard_normal((AMS_I, AM_D)) * 0.1).astype(np.float32)
        x_users = (rng.standard_normal((AMS_U, AM_D)) * 0.1).astype(np.float32)
        y_own, y_rep = sh.layer(torch.from_numpy(x_items[sh.u0:sh.u1]).to(dev), torch.from_numpy(x_users).to(dev))
        y1_own, y1_rep = sh.propagate(torch.from_numpy(x_items[sh.u0:sh.u1]).to(dev),
                                      torch.from_numpy(x_users).to(dev), 2)
        torch.cuda.synchronize()
        q.put((rank, sh.u0, sh.u1, y_own.cpu().numpy(), y_rep.cpu().numpy(), y1_own.cpu().numpy(),
               y1_rep.cpu().numpy()))
    except Exception:
        import traceback
        q.put((rank, 'error', traceback.format_exc(), None, None, None, None))
    finally:
        tdist.destroy_process_group()


def test_items_sharded_world2_one_gpu_matches_oracle():
    """BASELINE configuration 4's partition: items outnumber users (Amazon-Books-shaped,
    dataset.py:229-255), so the ITEMS are cut into ranges and the user block is
    replicated and all-reduced.  Two ranks on one GPU (gloo, host-staged), one layer
    and two chained layers, against the float64 oracle of D^-1/2 A D^-1/2."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_am_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
    for r in res:
        assert r[1] != 'error', r[2]
    pairs = _amazon_pairs()
    A = O.norm_adj(AMS_U, AMS_I, pairs)  # rows [users; items]
    rng = np.random.default_rng(3)
    x_items = (rng.standard_normal((AMS_I, AM_D)) * 0.1).astype(np.float32)
    x_users = (rng.standard_normal((AMS_U, AM_D)) * 0.1).astype(np.float32)
    x = np.concatenate([x_users, x_items])
    y = O.spmm64(A, x)
    y2 = _spmm64_f64(A, y)
    assert res[0][1] == 0 and res[-1][2] == AMS_I and res[0][2] == res[1][1]
    for rank, i0, i1, y_own, y_rep, y2_own, y2_rep in res:
        close(y_own, y[AMS_U + i0:AMS_U + i1], atol_row=2e-6)
        close(y_rep, y[:AMS_U], atol_row=2e-6)       # the replicated user block, all-reduced
        close(y2_own, y2[AMS_U + i0:AMS_U + i1], rtol=2e-5, atol_row=3e-6)
        close(y2_rep, y2[:AMS_U], rtol=2e-5, atol_row=3e-6)
    # both ranks hold the same reduced user block, bit for bit
    assert np.array_equal(res[0][4], res[1][4]) and np.array_equal(res[0][6], res[1][6])
