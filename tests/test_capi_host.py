"""C-ABI library (CPU-side): loads, exports every declared symbol, and its host
graph builders match the oracle / golden fixtures bit-exactly."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT
from igr import _lib
from igr import graph as G
from igr import model as M
from igr import ops
from oracle import igr_oracle as O


def declared_symbols():
    txt = open(os.path.join(ROOT, 'include', 'igr.h')).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(igr_[a-z0-9_]+)\s*\(', txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f'{s} declared in include/igr.h but not exported'
    assert set(syms) == set(_lib.SIGNATURES), 'ctypes binding out of sync with include/igr.h'
    assert lib.igr_version() == 10000


def test_binding_arity_matches_header():
    """Every prototype in include/igr.h has as many parameters as its ctypes
    argtypes entry (a parameter added to the C ABI but not to the binding would
    shift every later argument)."""
    txt = open(os.path.join(ROOT, 'include', 'igr.h')).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    protos = dict(re.findall(r'\b(igr_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;', txt, flags=re.S))
    assert len(protos) == len(_lib.SIGNATURES)
    for name, params in protos.items():
        params = params.strip()
        n = 0 if params in ('', 'void') else params.count(',') + 1
        assert n == len(_lib.SIGNATURES[name][1]), (name, n, len(_lib.SIGNATURES[name][1]))


def test_error_path_reports_message():
    with pytest.raises(_lib.IgrError, match='index out of range'):
        G.csr_from_coo(np.array([0, 5]), np.array([0, 0]), 3, 3)
    n = ctypes.c_int64()
    with pytest.raises(_lib.IgrError, match='chunk_edges'):
        _lib.call('igr_plan_size', 1, np.array([0, 1], np.int64).ctypes.data, 4, 100, ctypes.byref(n),
                  ctypes.byref(n), ctypes.byref(n))


def test_device_ops_refuse_cpu_tensors():
    rp, ci, v, _ = G.csr_from_coo(np.array([0, 1]), np.array([1, 0]), 2, 2)
    g = G.Graph(rp, ci, 2, 2, device='cpu')
    with pytest.raises(_lib.IgrError, match='no CPU fallback'):
        ops.spmm(g, torch.ones(2, 4))


@pytest.mark.parametrize('dedup', [True, False])
def test_csr_from_coo_matches_oracle(dedup):
    rng = np.random.default_rng(1)
    n_rows, n_cols, nnz = 300, 200, 5000
    row, col = rng.integers(0, n_rows, nnz), rng.integers(0, n_cols, nnz)
    val = rng.random(nnz).astype(np.float32)
    rp, ci, v, eid = G.csr_from_coo(row, col, n_rows, n_cols, val, dedup)
    ref = O.coo_to_csr(n_rows, n_cols, row, col, val, dedup)
    np.testing.assert_array_equal(rp, ref.row_ptr)
    np.testing.assert_array_equal(ci, ref.col)
    np.testing.assert_array_equal(v, ref.val)
    np.testing.assert_array_equal(eid, ref.eid)


def test_csr_transpose_matches_oracle():
    rng = np.random.default_rng(2)
    row, col = rng.integers(0, 50, 900), rng.integers(0, 70, 900)
    rp, ci, v, _ = G.csr_from_coo(row, col, 50, 70, None, True)
    t_rp, t_ci, t_pos = G.csr_transpose(rp, ci, 50, 70)
    A = O.CSR(50, 70, rp, ci.astype(np.int64), v)
    T = A.transpose()
    np.testing.assert_array_equal(t_rp, T.row_ptr)
    np.testing.assert_array_equal(t_ci, T.col)
    np.testing.assert_array_equal(t_pos, T.eid)


def test_plan_covers_rows_heaviest_first():
    rng = np.random.default_rng(3)
    deg = np.concatenate([rng.integers(0, 40, 500), [0, 0, 2000, 700, 5000, 513, 512]])
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    p = G.plan(rp, split_threshold=512, chunk_edges=256, window=0)
    order, sr, sp, cr, cb = p['order'], p['split_row'], p['split_ptr'], p['chunk_row'], p['chunk_beg']
    assert sorted(np.concatenate([order, sr]).tolist()) == list(range(len(deg)))
    assert np.all(deg[order] <= 512) and np.all(deg[sr] > 512)
    assert np.all(np.diff(deg[order]) <= 0) and np.all(np.diff(deg[sr]) <= 0)
    for s, r in enumerate(sr):
        chunks = list(range(sp[s], sp[s + 1]))
        assert all(cr[c] == r for c in chunks)
        np.testing.assert_array_equal(cb[chunks], np.arange(rp[r], rp[r + 1], 256))
    # windowed: each window of 100 rows is a degree-descending run, windows in row order
    pw = G.plan(rp, split_threshold=512, chunk_edges=256, window=100)
    ow = pw['order']
    assert sorted(ow.tolist()) == sorted(order.tolist())
    win = ow // 100
    assert np.all(np.diff(win) >= 0)
    for w in np.unique(win):
        assert np.all(np.diff(deg[ow[win == w]]) <= 0)
    np.testing.assert_array_equal(pw['split_row'], sr)


def test_norm_adj_host_build_bit_exact(golden):
    nu, ni = int(golden['n_users']), int(golden['n_items'])
    g, vals, deg, dinv = M.build_norm_adj(nu, ni, golden['train_array'], 'cpu')
    h = g.host()
    np.testing.assert_array_equal(np.repeat(np.arange(nu + ni), np.diff(h['row_ptr'])), golden['norm_idx'][0])
    np.testing.assert_array_equal(h['col_idx'], golden['norm_idx'][1])
    np.testing.assert_array_equal(deg, golden['degree'])
    np.testing.assert_array_equal(dinv, golden['dinv'])
    np.testing.assert_array_equal(vals.numpy(), golden['norm_val'])


def test_feat_structure_bit_exact(golden):
    nu, ni = int(golden['n_users']), int(golden['n_items'])
    ta = golden['train_array']
    F = O.generate_feat(nu, ni, ta)
    U, I = nu, ni
    u, i = ta[:, 0], ta[:, 1]
    row = np.concatenate([u, U + i, np.arange(U), U + np.arange(I)])
    col = np.concatenate([U + i, u, np.full(U, U + I), np.full(I, U + I + 1)])
    rp, ci, v, _ = G.csr_from_coo(row, col, U + I, U + I + 2, None, True)
    np.testing.assert_array_equal(np.repeat(np.arange(U + I), np.diff(rp)), golden['feat_idx'][0])
    np.testing.assert_array_equal(ci, golden['feat_idx'][1])
    np.testing.assert_array_equal(G.row_sums(rp, v), golden['row_sum'])
    np.testing.assert_array_equal(G.row_sums(rp, v), F.row_sum)


def test_reverse_graph_edge_ids():
    rng = np.random.default_rng(4)
    src, dst = rng.integers(0, 30, 400), rng.integers(0, 20, 400)
    g = ops.graph((torch.from_numpy(src), torch.from_numpy(dst)), num_nodes=30, device='cpu')
    h = g.host()
    assert h['edge_id'] is not None
    rows = np.repeat(np.arange(30), np.diff(h['row_ptr']))
    # CSR position p holds input edge edge_id[p]: dst == row, src == col
    np.testing.assert_array_equal(dst[h['edge_id']], rows)
    np.testing.assert_array_equal(src[h['edge_id']], h['col_idx'])
    r = g.reverse()
    rh = r.host()
    rrows = np.repeat(np.arange(30), np.diff(rh['row_ptr']))
    np.testing.assert_array_equal(src[rh['edge_id']], rrows)
    np.testing.assert_array_equal(dst[rh['edge_id']], rh['col_idx'])
    # the positional view: same arrays, schedule and workspaces, per-edge data read by CSR position
    p = r.positional()
    assert p is r.positional() and p.edge_id is None and not p.csr.edge_id and r.csr.edge_id
    assert p.csr.row_ptr == r.csr.row_ptr and p.csr.col_idx == r.csr.col_idx and p.csr.n_chunks == r.csr.n_chunks
    assert p._ws is r._ws
    # the reverse of a positional view addresses per-edge data by the VIEW's order (CSR position
    # of r), not by the input edge ids: with the values permuted once, it rebuilds the same matrix
    pv = rng.standard_normal(400).astype(np.float32)          # values by input edge id
    pos_vals = pv[rh['edge_id']]                              # ... permuted into r's CSR order
    pr = p.reverse()
    assert pr is p.reverse() and pr is not r.reverse()
    prh = pr.host()
    dense = np.zeros((pr.n_rows, pr.n_cols), np.float64)
    np.add.at(dense, (np.repeat(np.arange(pr.n_rows), np.diff(prh['row_ptr'])), prh['col_idx']),
              pos_vals[prh['edge_id']])
    want = np.zeros_like(dense)
    np.add.at(want, (dst, src), pv)                           # g: rows = dst, cols = src
    np.testing.assert_allclose(dense, want, rtol=0, atol=1e-12)
    # values permuted once (vals[edge_id]) then read in order = values read through the edge ids
    vals = rng.standard_normal(400).astype(np.float32)
    np.testing.assert_array_equal(vals[rh['edge_id']][np.arange(r.nnz)], vals[rh['edge_id']])
    plain = ops.graph((torch.arange(5), torch.arange(5)), num_nodes=5, device='cpu')
    assert plain.positional() is plain  # no edge-id permutation: the graph itself


def _refused(name, *args, match=None):
    """The call must fail argument validation (before any device work) with IGR_ERR_ARG."""
    rc = getattr(_lib.lib(), name)(*args)
    assert rc == 1, (name, rc)
    if match:
        msg = _lib.lib().igr_last_error().decode()
        assert re.search(match, msg), msg


def test_new_entry_points_validate_arguments():
    """Argument checks of the batch-row, pull, top-k, split-K GEMM, BPR and fused-dropout
    entry points run on the host: wrong shapes are refused with IGR_ERR_ARG and a message."""
    F = ctypes.c_void_p(0x10000)  # 16-B aligned stand-in device pointer, never dereferenced here
    rp, ci, _, eid = G.csr_from_coo(np.array([0, 1, 1]), np.array([1, 0, 2]), 2, 3, dedup=False)
    rect = G.Graph(rp, ci, 2, 3, device='cpu')  # 2 x 3
    multi = G.Graph(rp, ci, 2, 3, device='cpu', edge_id=eid[::-1].copy())
    st = None
    # top-k: k in [1, 1024] and <= n_cols; ld >= n_cols
    _refused('igr_topk_f32', 2, 5, F, 5, 6, F, F, st, match='k larger')
    _refused('igr_topk_f32', 2, 5, F, 5, 0, F, F, st, match=r'\[1, 1024\]')
    _refused('igr_topk_f32', 2, 5000, F, 5000, 2000, F, F, st, match=r'\[1, 1024\]')
    _refused('igr_topk_f32', 2, 5, F, 4, 2, F, F, st, match='ld')
    _refused('igr_mask_scores_f32', 2, None, None, F, 5, st, match='NULL')
    # GEMM: sizes / leading dims; the split-K workspace is asked for only where it is used
    _refused('igr_gemm_f32', -1, 4, 4, F, 4, 0, F, 4, 0, None, F, 4, None, 0, st, match='negative')
    _refused('igr_gemm_f32', 8, 8, 8, F, 8, 0, F, 8, 0, None, F, 4, None, 0, st, match='ldc')
    assert _lib.lib().igr_gemm_workspace_size(256, 64, 9750) > 0  # weight gradient: split K
    assert _lib.lib().igr_gemm_workspace_size(100000, 64, 64) == 0  # tall: no split
    # row-restricted SpMM / push / pull
    _refused('igr_spmm_rows_f32', ctypes.byref(rect.csr), 48, F, 4, F, 48, None, None, 0, None, 0, 1.0, F, 48, st,
             match='d must be')
    _refused('igr_spmm_rows_f32', ctypes.byref(multi.csr), 64, F, 4, F, 64, F, None, 0, None, 0, 1.0, F, 64, st,
             match='edge_id')
    tall = G.Graph(np.array([0, 1, 2, 3]), np.array([0, 1, 0], np.int32), 3, 2, device='cpu')  # 3 x 2
    _refused('igr_spmm_push_f32', ctypes.byref(tall.csr), 64, F, 4, F, 64, None, 1.0, 1, F, 64, st, match='square')
    _refused('igr_spmm_pull_marked_f32', ctypes.byref(rect.csr), 64, None, F, F, F, 64, None, 1.0, 0, None, F, 64, st,
             match='NULL')
    _refused('igr_spmm_pull_marked_f32', ctypes.byref(multi.csr), 64, F, F, F, F, 64, F, 1.0, 0, None, F, 64, st,
             match='edge_id')
    # the shard set-up passes (host memory): sizes, pointers and the output pair are checked
    n_out = ctypes.c_int64(0)
    _refused('igr_count_ids', -1, None, 4, None, 0, match='bad args')
    _refused('igr_count_ids', 3, None, 4, None, 0, match='bad args')
    _refused('igr_select_id_range', 3, None, None, 0, 2, None, None, ctypes.byref(n_out), 0, match='bad args')
    keys = np.array([0, 1, 2], np.int64)
    _refused('igr_select_id_range', 3, keys.ctypes.data, None, 0, 2, keys.ctypes.data, None, ctypes.byref(n_out), 0,
             match='go together')
    _refused('igr_rowset_mark', 4, F, None, F, st, match='NULL')
    _refused('igr_rowset_sum_f32', 4, 64, F, F, 32, 1.0, F, F, 64, st, match='leading')
    _refused('igr_rowset_sum_f32', 4, 64, None, F, 64, 1.0, F, F, 64, st, match='NULL')
    # fixed-order accumulation: the sort needs its key buffer, the scatter its sorted keys
    _refused('igr_rowsort', 4, F, 0, None, 0, F, 0, F, st, match='idx2 without idx1')
    _refused('igr_rowsort', 4, F, 0, None, 0, None, 0, None, st, match='NULL')
    _refused('igr_scatter_add_rows_f32', 4, 64, None, F, 64, F, 64, st, match='NULL')
    assert _lib.lib().igr_rowsort_size(0) == 0
    assert _lib.lib().igr_rowsort_size(6144) == 2 * 6144      # 6 tiles of 1024, ranked in one pass
    assert _lib.lib().igr_rowsort_size(1000) == 2 * 1024
    assert _lib.lib().igr_rowsort_size(100 * 1024) == 2 * 128 * 1024  # > 64 tiles: padded to a power of two
    # fused BPR: the backward needs its workspace; fused dropout: keep in (0, 1]
    assert _lib.lib().igr_bpr_workspace_floats(2048, 64) == 3 * 2048 * 64 + 128 * 64
    _refused('igr_bpr_fwd_bwd_f32', 4, 64, F, F, F, 0, 0, F, 64, F, None, None, 1.0, 0.0, None, None, F, 64,
             None, F, None, st, match='workspace')
    for keep in (0.0, 1.5):
        _refused('igr_spmm_scaled_f32', ctypes.byref(rect.csr), 64, F, 64, None, None, keep, 1, 0, None, 0, F, 64,
                 None, F, st, match='keep')
    _refused('igr_dropout_uniforms', None, 1, 0, None, 0, F, st, match='NULL')
    _refused('igr_edge_dropout_counter_f32', ctypes.byref(rect.csr), F, 1.0, 1, 0, None, 0, F, st, match='p must')
    # hipGraph-step entry points: the device counter, Adam's host step without one, per-head SpMM
    _refused('igr_counter_add', None, 1, st, match='NULL')
    _refused('igr_adam_multi_f32', 17, F, 1e-3, 0.9, 0.999, 1e-8, 0.0, None, st, match='n_slots')
    _refused('igr_adam_multi_f32', 1, None, 1e-3, 0.9, 0.999, 1e-8, 0.0, None, st, match='NULL')
    _refused('igr_means_f32', 0, F, None, F, st, match='n <= 0')
    assert _lib.lib().igr_linear_wgrad_workspace_size(1000, 192, 64) == 0      # 3 blocks of 64: the GEMM takes it
    assert _lib.lib().igr_linear_wgrad_workspace_size(1_100_002, 256, 64) == 256 * 256 * 65 * 4   # 1024 waves / 4 blocks
    _refused('igr_linear_wgrad_f32', 1000, 100, 64, F, 100, F, 64, F, 64, None, F, 1 << 20, st, match='supported')
    _refused('igr_linear_wgrad_f32', 1000, 64, 64, F, 64, F, 64, F, 64, None, None, 0, st, match='workspace')
    _refused('igr_loss_combine_f32', None, None, None, 0.0, 0.0, 1.0, F, None, st, match='bpr')
    _refused('igr_adam_f32', 4, F, F, F, F, 1e-3, 0.9, 0.999, 1e-8, 0.0, 0, None, st, match='step')
    _refused('igr_bpr_sample', 4, 0, F, F, F, 10, 1, 0, None, 8, F, F, F, st, match='active')
    _refused('igr_spmm_heads_f32', ctypes.byref(rect.csr), 4, 64, F, 64, F, F, 256, None, st, match='leading')
    # one value per node: graph and pointers
    _refused('igr_spmv_f32', None, F, None, F, st, match='NULL')
    _refused('igr_spmv_f32', ctypes.byref(rect.csr), F, None, None, st, match='NULL')
    # NGCF's layer tail: width and leading dimensions
    _refused('igr_layer_tail_f32', 4, 300, F, 300, F, 300, None, 1.0, 0.2, F, F, 300, F, st, match='d <= 256')
    _refused('igr_layer_tail_f32', 4, 64, F, 32, F, 64, None, 1.0, 0.2, F, F, 64, F, st, match='leading')
    _refused('igr_layer_tail_f32', 4, 64, F, 64, F, 64, None, 1.0, 0.2, F, None, 64, F, st, match='NULL')
    _refused('igr_layer_tail_bwd_f32', 4, 64, F, 32, None, 0, F, F, None, 1.0, 0.2, F, st, match='leading')
    _refused('igr_layer_tail_bwd_f32', 4, 64, F, 64, None, 0, F, None, None, 1.0, 0.2, F, st, match='NULL')
    assert _lib.lib().igr_layer_tail_f32(0, 64, None, 64, None, 64, None, 1.0, 0.2, None, None, 64, None, st) == 0
    assert _lib.lib().igr_linear_wgrad_workspace_size(70839, 512, 128) > 0  # the d = 128 projections


def test_shared_heads_workspace_contract():
    """igr_spmm_shared_heads_ws_f32: the workspace holds one h * d partial per chunk of the
    graph's split rows (none when no row is split); a smaller or misaligned one is refused."""
    F = ctypes.c_void_p(0x10000)
    rp = np.array([0, 700, 705, 2000], np.int64)
    ci = np.zeros(2000, np.int32)
    cut = G.Graph(rp, ci, 3, 8, device='cpu', split_threshold=128, chunk_edges=256)
    whole = G.Graph(rp, ci, 3, 8, device='cpu', split_threshold=1 << 30, chunk_edges=1 << 30)
    assert (cut.n_split, cut.n_chunks, whole.n_chunks) == (2, 3 + 6, 0)
    size = _lib.lib().igr_spmm_shared_heads_workspace_size
    assert size(ctypes.byref(cut.csr), 4, 64) == 9 * 4 * 64 * 4
    assert size(ctypes.byref(whole.csr), 4, 64) == 0 and size(None, 4, 64) == 0
    _refused('igr_spmm_shared_heads_ws_f32', ctypes.byref(cut.csr), 4, 64, F, 64, F, F, 256, F, 9 * 4 * 64 * 4 - 1, None,
             match='workspace smaller')
    _refused('igr_spmm_shared_heads_ws_f32', ctypes.byref(cut.csr), 4, 64, F, 64, F, F, 256, ctypes.c_void_p(0x10004),
             9 * 4 * 64 * 4, None, match='16-byte')
    _refused('igr_spmm_shared_heads_ws_f32', ctypes.byref(cut.csr), 3, 64, F, 64, F, F, 256, F, 1 << 20, None,
             match='supported')
    # the edge softmax by chunks: 2 h floats per chunk forward, h backward
    ssize = _lib.lib().igr_att_softmax_workspace_size
    assert ssize(ctypes.byref(cut.csr), 4) == 9 * 8 * 4 and ssize(ctypes.byref(whole.csr), 4) == 0
    _refused('igr_att_softmax_ws_f32', ctypes.byref(cut.csr), 4, F, None, 8.0, F, F, F, F, 9 * 8 * 4 - 1, None,
             match='workspace smaller')
    _refused('igr_att_softmax_bwd_ws_f32', ctypes.byref(cut.csr), 4, F, None, 8.0, F, F, F, F, F, 9 * 4 * 4 - 1, None,
             match='workspace smaller')
    _refused('igr_att_softmax_bwd_ws_f32', ctypes.byref(cut.csr), 4, F, None, 8.0, None, F, F, F, F, 1 << 20, None,
             match='row_max')


def test_auto_plan_is_a_function_of_the_degrees():
    """igr.graph.auto_plan: the default plan for graphs of alike rows and for graphs above
    4 M edges; a lower split threshold when a few rows are far longer than the rest; the
    same answer for the same degrees (runs stay bitwise reproducible)."""
    rng = np.random.default_rng(0)
    alike = np.concatenate([[0], np.cumsum(rng.integers(150, 330, 9746))])
    assert G.auto_plan(alike) == (512, 512)
    deg = rng.integers(20, 200, 9746)
    deg[:300] = rng.integers(600, 4000, 300)  # hub rows
    skew = np.concatenate([[0], np.cumsum(deg)])
    t, c = G.auto_plan(skew)
    assert t < 512 and c == min(2 * t, 512) and G.auto_plan(skew.copy()) == (t, c)
    big = np.concatenate([[0], np.cumsum(np.full(30000, 200))])  # 6 M edges
    assert G.auto_plan(big) == (512, 512)
    short = np.concatenate([[0], np.cumsum(rng.integers(0, 60, 5000))])  # nothing to split
    assert G.auto_plan(short) == (512, 512)
    g = G.Graph(skew, np.zeros(int(skew[-1]), np.int32), len(deg), 1, device='cpu')
    assert (g.split_threshold, g.chunk_edges) == (t, c) and g.n_split > 0
    assert G.Graph(skew, np.zeros(int(skew[-1]), np.int32), len(deg), 1, device='cpu', split_threshold=512,
                   chunk_edges=512).split_threshold == 512
