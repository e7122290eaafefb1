"""Graph: a CSR graph resident in HBM plus its row schedule.

Replaces the per-call `dgl.graph((column, row), num_nodes=..., device=...)`
of the reference (model.py:103-105, 4183, 4194): the structure is built once
on the host (C++ in libigr, include/igr.h) and kept on the device; only edge
values change between steps (dropout, anneal).

Layout in HBM:
    row_ptr  int64[n_rows+1]   col_idx int32[nnz]   edge_id int64[nnz] | None
    order    int32[n_order]    rows of degree <= split_threshold, heaviest first
    split_row int32, split_ptr int64, chunk_row int32, chunk_beg int64  (long rows)
"""
import copy
import ctypes

import numpy as np
import torch

from . import _lib as L

DEFAULT_SPLIT_THRESHOLD = 512
DEFAULT_CHUNK_EDGES = 512
DEFAULT_WINDOW = 65536  # degree-sort window (rows); 0 = global


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data if a.size else None
    return a.data_ptr() if a.numel() else None


def _np(a, dt):
    if isinstance(a, torch.Tensor):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(a, dtype=dt)


# ------------------------------------------------------------------ host builders (C++)

def csr_from_coo(row, col, n_rows, n_cols, val=None, dedup=True, n_threads=0, want_eid=True):
    """COO -> CSR sorted by (row, col).  dedup sums duplicates (scipy .tocsr() +
    torch .coalesce(), utils.py:33-50); otherwise every edge is kept and
    `edge_id` maps CSR position -> input edge index (DGL edge id)."""
    row, col = _np(row, np.int64), _np(col, np.int64)
    v = None if val is None else _np(val, np.float32)
    nnz = len(row)
    row_ptr = np.empty(n_rows + 1, np.int64)
    col_idx = np.empty(max(nnz, 1), np.int32)
    val_out = np.empty(max(nnz, 1), np.float32)
    eid = np.empty(max(nnz, 1), np.int64) if want_eid else None
    n = ctypes.c_int64(0)
    L.call('igr_csr_from_coo', n_rows, n_cols, nnz, _ptr(row), _ptr(col), _ptr(v), int(bool(dedup)),
           _ptr(row_ptr), _ptr(col_idx), _ptr(val_out), _ptr(eid), ctypes.byref(n), n_threads)
    k = n.value
    return row_ptr, col_idx[:k].copy(), val_out[:k].copy(), None if eid is None else eid[:k].copy()


def count_ids(ids, n_bins, n_threads=0):
    """int64[n_bins]: occurrences of each id (np.bincount, multi-threaded)."""
    ids = _np(ids, np.int64)
    out = np.empty(n_bins, np.int64)
    L.call('igr_count_ids', len(ids), _ptr(ids), n_bins, _ptr(out), n_threads)
    return out


def select_id_range(key, other, lo, hi, n_threads=0):
    """(key - lo, other) for the pairs with lo <= key < hi, in input order."""
    key, other = _np(key, np.int64), _np(other, np.int64)
    assert len(key) == len(other)
    n = ctypes.c_int64(0)
    L.call('igr_select_id_range', len(key), _ptr(key), _ptr(other), lo, hi, None, None, ctypes.byref(n), n_threads)
    ok, oo = np.empty(n.value, np.int64), np.empty(n.value, np.int64)
    if n.value:
        L.call('igr_select_id_range', len(key), _ptr(key), _ptr(other), lo, hi, _ptr(ok), _ptr(oo), ctypes.byref(n),
               n_threads)
    return ok, oo


def csr_transpose(row_ptr, col_idx, n_rows, n_cols, n_threads=0):
    """Reverse graph: (t_row_ptr, t_col_idx, t_pos) with t_pos = forward CSR position."""
    row_ptr, col_idx = _np(row_ptr, np.int64), _np(col_idx, np.int32)
    nnz = int(row_ptr[-1])
    t_rp = np.empty(n_cols + 1, np.int64)
    t_ci = np.empty(max(nnz, 1), np.int32)
    t_pos = np.empty(max(nnz, 1), np.int64)
    L.call('igr_csr_transpose', n_rows, n_cols, _ptr(row_ptr), _ptr(col_idx), _ptr(t_rp), _ptr(t_ci),
           _ptr(t_pos), n_threads)
    return t_rp, t_ci[:nnz], t_pos[:nnz]


def row_sums(row_ptr, val=None):
    row_ptr = _np(row_ptr, np.int64)
    v = None if val is None else _np(val, np.float32)
    out = np.empty(len(row_ptr) - 1, np.float32)
    L.call('igr_csr_row_sums', len(row_ptr) - 1, _ptr(row_ptr), _ptr(v), _ptr(out))
    return out


def sym_norm_values(row_ptr, col_idx, val, dinv, dinv_col=None):
    """(dinv[r] * val) * dinv_col[c]  (model.py:91-96); dinv_col defaults to dinv."""
    row_ptr, col_idx = _np(row_ptr, np.int64), _np(col_idx, np.int32)
    v = None if val is None else _np(val, np.float32)
    dinv = _np(dinv, np.float32)
    dc = dinv if dinv_col is None else _np(dinv_col, np.float32)
    out = np.empty(len(col_idx), np.float32)
    L.call('igr_sym_norm_values', len(row_ptr) - 1, _ptr(row_ptr), _ptr(col_idx), _ptr(v), _ptr(dinv), _ptr(dc),
           _ptr(out))
    return out


def plan(row_ptr, split_threshold=DEFAULT_SPLIT_THRESHOLD, chunk_edges=DEFAULT_CHUNK_EDGES, window=None):
    """Degree-binned row schedule (see include/igr.h igr_plan_fill)."""
    row_ptr = _np(row_ptr, np.int64)
    n_rows = len(row_ptr) - 1
    no, ns, nc = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    L.call('igr_plan_size', n_rows, _ptr(row_ptr), split_threshold, chunk_edges,
           ctypes.byref(no), ctypes.byref(ns), ctypes.byref(nc))
    order = np.empty(max(no.value, 1), np.int32)
    split_row = np.empty(max(ns.value, 1), np.int32)
    split_ptr = np.empty(ns.value + 1, np.int64)
    chunk_row = np.empty(max(nc.value, 1), np.int32)
    chunk_beg = np.empty(max(nc.value, 1), np.int64)
    window = DEFAULT_WINDOW if window is None else window
    L.call('igr_plan_fill', n_rows, _ptr(row_ptr), split_threshold, chunk_edges, window, _ptr(order),
           _ptr(split_row), _ptr(split_ptr), _ptr(chunk_row), _ptr(chunk_beg))
    return dict(order=order[:no.value], split_row=split_row[:ns.value], split_ptr=split_ptr,
                chunk_row=chunk_row[:nc.value], chunk_beg=chunk_beg[:nc.value], chunk_edges=chunk_edges)


# Row-plan choice for small graphs.  On a graph whose rows all run at once (a few thousand to
# a few tens of thousands of rows) an SpMM lasts as long as its longest unsplit row: one
# 16-lane group walks that row 16 edges per round, ~1.6 us a round on MI355X, while the
# split rows' chunks (one wave each) and the combine pass cost a few us in total.  The
# estimate below was fitted to measured launches (ML-100K / ML-1M shapes, uniform and
# MovieLens-like item popularity, 7 thresholds each; scripts/tune_small_plan.py) and is
# evaluated on the degree array alone, so a graph always gets the same plan.
AUTO_PLAN_MAX_NNZ = 4_000_000  # larger graphs are throughput-bound: the default plan
_PLAN_THRESHOLDS = (512, 384, 256, 192, 128, 96, 64)


def auto_plan(row_ptr):
    """(split_threshold, chunk_edges) for this degree distribution."""
    deg = np.diff(_np(row_ptr, np.int64))
    if len(deg) == 0 or int(row_ptr[-1]) > AUTO_PLAN_MAX_NNZ or int(deg.max()) <= _PLAN_THRESHOLDS[-1]:
        return DEFAULT_SPLIT_THRESHOLD, DEFAULT_CHUNK_EDGES
    best = None
    for t in _PLAN_THRESHOLDS:  # ties go to the larger threshold (fewer split rows)
        c = min(2 * t, DEFAULT_CHUNK_EDGES)
        fast, split = deg[deg <= t], deg[deg > t]
        rounds = -(-int(fast.max()) // 16) if fast.size else 0
        chunk_rounds = -(-min(c, int(split.max())) // 64) if split.size else 0
        est = max(1.57 * rounds, 16.1e-6 * float(fast.sum()), 0.8 * chunk_rounds)
        if split.size:
            est += 3.29e-6 * float(split.sum()) + 1.96e-3 * split.size + 0.38e-3 * float((-(-split // c)).sum()) + 2.8
        if best is None or est < best[0]:
            best = (est, t, c)
    return best[1], best[2]


# ------------------------------------------------------------------ Graph

class Graph:
    """CSR over destination rows; columns are source nodes.

    `rhs` edge data passed to the ops is indexed by edge id, which equals the
    CSR position unless `edge_id` is given (DGL multigraph built from an
    unsorted edge list)."""

    def __init__(self, row_ptr, col_idx, n_rows, n_cols, device='cuda', edge_id=None, symmetric=False,
                 split_threshold=None, chunk_edges=None, window=None):
        row_ptr = _np(row_ptr, np.int64)
        col_idx = _np(col_idx, np.int32)
        # no plan given: chosen from the degree distribution (auto_plan)
        self._auto_plan = split_threshold is None and chunk_edges is None
        if self._auto_plan:
            split_threshold, chunk_edges = auto_plan(row_ptr)
        split_threshold = DEFAULT_SPLIT_THRESHOLD if split_threshold is None else split_threshold
        chunk_edges = DEFAULT_CHUNK_EDGES if chunk_edges is None else chunk_edges
        self.n_rows, self.n_cols = int(n_rows), int(n_cols)
        assert len(row_ptr) == self.n_rows + 1, 'row_ptr must have n_rows + 1 entries'
        self.nnz = int(row_ptr[-1])
        assert len(col_idx) == self.nnz
        self.max_row_edges = int(np.diff(row_ptr).max()) if self.n_rows else 0
        if edge_id is not None:
            edge_id = _np(edge_id, np.int64)
            if np.array_equal(edge_id, np.arange(self.nnz, dtype=np.int64)):
                edge_id = None
        self.device = torch.device(device)
        self.symmetric = symmetric
        self.split_threshold, self.chunk_edges = split_threshold, chunk_edges
        self._host = dict(row_ptr=row_ptr, col_idx=col_idx, edge_id=edge_id)
        p = plan(row_ptr, split_threshold, chunk_edges, window)
        self.window = window
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)  # noqa: E731
        self.row_ptr = t(row_ptr)
        self.col_idx = t(col_idx)
        self.edge_id = None if edge_id is None else t(edge_id)
        self.order = t(p['order'])
        self.split_row = t(p['split_row'])
        self.split_ptr = t(p['split_ptr'])
        self.chunk_row = t(p['chunk_row'])
        self.chunk_beg = t(p['chunk_beg'])
        self.n_order, self.n_split, self.n_chunks = len(p['order']), len(p['split_row']), len(p['chunk_row'])
        self.csr = L.IgrCsr(
            self.n_rows, self.n_cols, self.nnz, _ptr(self.row_ptr), _ptr(self.col_idx), _ptr(self.edge_id),
            self.n_order, _ptr(self.order), self.n_split, _ptr(self.split_row), _ptr(self.split_ptr),
            self.n_chunks, _ptr(self.chunk_row), _ptr(self.chunk_beg), chunk_edges)
        self._reverse = self if symmetric else None
        self._ws = {}
        self._edge_rows = None

    # -- constructors
    @classmethod
    def from_coo(cls, row, col, n_rows, n_cols, val=None, dedup=True, device='cuda', **kw):
        """Returns (graph, values-by-edge-id as float32 numpy)."""
        rp, ci, v, eid = csr_from_coo(row, col, n_rows, n_cols, val, dedup)
        g = cls(rp, ci, n_rows, n_cols, device=device, edge_id=None if dedup else eid, **kw)
        if not dedup:
            # values are addressed by edge id: scatter back to input order
            vv = np.empty(len(eid), np.float32)
            vv[eid] = v
            v = vv
        return g, v

    values = None  # float32[nnz] by edge id when the graph carries its edge values (model.norm_adj)

    def with_values(self, values):
        """This graph with another set of edge values - what the reference holds as a
        second sparse tensor over the same indices (NGCF.dropout_sp_mat, model.py:4016-4028).
        A view: device arrays, schedule, workspaces and the reverse graph stay the base graph's."""
        g = copy.copy(self)
        g._base = getattr(self, '_base', None) or self
        g.values = values
        return g

    def positional(self):
        """This graph reading per-edge arrays by CSR position instead of by edge id (a view:
        a caller that has permuted its values once, `values[g.edge_id]`, then reads them in
        stream order in every product over this graph)."""
        if self.edge_id is None:
            return self
        v = self.__dict__.get('_positional')
        if v is None:
            v = copy.copy(self)
            v._base = getattr(self, '_base', None) or self
            v.edge_id = None
            v.csr = L.IgrCsr.from_buffer_copy(self.csr)
            v.csr.edge_id = None
            self._positional = v
        return v

    def reverse(self):
        """Reverse graph for gspmm backward; its edge ids are this graph's edge ids."""
        base = getattr(self, '_base', None)
        if base is not None:
            if self.edge_id is None and base.edge_id is not None:
                # a positional view: its per-edge arrays are in this graph's CSR order, so the
                # reverse must address them by forward CSR position (t_pos), not by the base
                # graph's edge ids
                rev = self.__dict__.get('_pos_reverse')
                if rev is None:
                    h = base._host
                    t_rp, t_ci, t_pos = csr_transpose(h['row_ptr'], h['col_idx'], self.n_rows, self.n_cols)
                    own = {} if base._auto_plan else dict(split_threshold=base.split_threshold,
                                                          chunk_edges=base.chunk_edges)
                    rev = Graph(t_rp, t_ci, self.n_cols, self.n_rows, device=self.device, edge_id=t_pos, **own)
                    self._pos_reverse = rev
                return rev
            return base.reverse()
        if self._reverse is None:
            h = self._host
            t_rp, t_ci, t_pos = csr_transpose(h['row_ptr'], h['col_idx'], self.n_rows, self.n_cols)
            eid = t_pos if h['edge_id'] is None else h['edge_id'][t_pos]
            own = {} if self._auto_plan else dict(split_threshold=self.split_threshold, chunk_edges=self.chunk_edges)
            self._reverse = Graph(t_rp, t_ci, self.n_cols, self.n_rows, device=self.device, edge_id=eid, **own)
            self._reverse._reverse = self
        return self._reverse

    def workspace(self, d):
        """Chunk partial sums for split rows (n_chunks * d floats), cached per d."""
        if self.n_chunks == 0:
            return None
        ws = self._ws.get(d)
        if ws is None:
            ws = torch.empty(self.n_chunks * d, dtype=torch.float32, device=self.device)
            self._ws[d] = ws
        return ws

    def edge_rows(self):
        """int64[nnz]: destination row of every edge, in edge-id order."""
        if self._edge_rows is None:
            h = self._host
            rows = np.repeat(np.arange(self.n_rows, dtype=np.int64), np.diff(h['row_ptr']))
            if h['edge_id'] is not None:
                r2 = np.empty_like(rows)
                r2[h['edge_id']] = rows
                rows = r2
            self._edge_rows = torch.from_numpy(rows).to(self.device)
        return self._edge_rows

    def host(self):
        return self._host

    def degrees(self):
        return np.diff(self._host['row_ptr'])

    def __repr__(self):
        return (f'Graph(n_rows={self.n_rows}, n_cols={self.n_cols}, nnz={self.nnz}, split_rows={self.n_split}, '
                f'chunks={self.n_chunks}, device={self.device})')


class TiledGraph:
    """A graph cut into source-column tiles: A = [A_0 | A_1 | ... ] by column range.

    y = sum_t A_t x[cols_t] is computed tile by tile, accumulating in place,
    so each pass gathers from a table slice small enough to stay resident in
    the Infinity Cache instead of streaming the whole source table from HBM.
    Pays off when the gathered table is much larger than the output
    (the item side of a user x item graph).  `perm` maps each tile's edge
    positions to positions of the parent CSR (to slice edge values)."""

    def __init__(self, parent_host, n_rows, n_cols, bounds, device, **kw):
        rp, ci = parent_host['row_ptr'], parent_host['col_idx']
        nnz = int(rp[-1])
        rows = np.repeat(np.arange(n_rows, dtype=np.int64), np.diff(rp))
        tile = np.searchsorted(np.asarray(bounds[1:-1], np.int64), ci, side='right').astype(np.int16)
        order = np.argsort(tile, kind='stable')  # edges grouped by tile, CSR order within a tile
        counts = np.bincount(tile, minlength=len(bounds) - 1)
        self.tiles, self.perms, self.bounds = [], [], list(bounds)
        start = 0
        for t in range(len(bounds) - 1):
            sel = order[start:start + counts[t]]
            start += counts[t]
            trp = np.concatenate([[0], np.cumsum(np.bincount(rows[sel], minlength=n_rows))]).astype(np.int64)
            tci = (ci[sel] - bounds[t]).astype(np.int32)
            self.tiles.append(Graph(trp, tci, n_rows, bounds[t + 1] - bounds[t], device=device, **kw))
            self.perms.append(torch.from_numpy(sel).to(device))
        self.n_rows, self.n_cols, self.nnz = n_rows, n_cols, nnz

    def tile_values(self, vals):
        """Per-tile contiguous value arrays (gathered once; values by parent CSR position)."""
        return [vals[p].contiguous() for p in self.perms]
