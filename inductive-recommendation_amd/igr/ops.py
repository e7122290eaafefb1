"""igr.ops - device operators of the inductive graph-convolution path.

Thin wrappers over the HIP C ABI (include/igr.h) and the autograd Functions
built from them.  PyTorch only provides device memory, the current stream
and autograd bookkeeping; every hot-path byte is moved by the HIP kernels.
Ops raise IgrError for tensors that are not on a ROCm device (no CPU
fallback).

DGL-compatible surface (the reference's operator API):
    graph((src, dst), num_nodes, device)       ~ dgl.graph       model.py:103-105
    gspmm(g, 'mul', 'sum', lhs, rhs)           ~ dgl.ops.gspmm   model.py:106, 4184, 4196, 4037
    gspmm(g, 'copy_rhs', 'sum'|'max', None, e) ~ dgl.ops.gspmm   model.py:4270, 4273
    gsddmm(g, 'dot', lhs, rhs)                 ~ AttIGCN.masked_mm model.py:4246-4255
"""
import ctypes
import weakref
import math

import numpy as np
import torch

from . import _lib as L
from .graph import Graph

IgrError = L.IgrError


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _written(out, fresh):
    """A kernel wrote `out` through its raw pointer: tell autograd's version counter when the
    buffer is the caller's (a value buffer reused across steps), so anything keyed on
    tensor._version - the permuted-values cache of the gspmm backward - sees the write."""
    if not fresh:
        torch.autograd.graph.increment_version(out)
    return out


def _dev(*ts):
    for t in ts:
        if t is not None and not (isinstance(t, torch.Tensor) and t.is_cuda):
            raise IgrError('igr device ops need tensors on a ROCm (HIP) device; got '
                           f'{t.device if isinstance(t, torch.Tensor) else type(t)}. There is no CPU fallback.')


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _f32(t):
    if t.dtype != torch.float32:
        raise IgrError(f'expected float32, got {t.dtype}')
    return t


def _rows(t):
    """2-D float32 with unit inner stride; returns (tensor, leading dim)."""
    _f32(t)
    if t.dim() != 2:
        raise IgrError('expected a 2-D tensor')
    if t.stride(1) != 1 or t.stride(0) < t.shape[1]:
        t = t.contiguous()
    return t, t.stride(0)


# ------------------------------------------------------------------ raw ops

def epilogue(alpha=1.0, beta=0.0, add=None, acc=None, acc_mode=0, acc_div=1.0, skip_y=False, row_scale=None,
             row_mask=None, col_mask=None):
    """struct igr_epilogue for spmm / spmm_scaled.  The struct holds raw device
    pointers, so it also keeps the tensors alive (an inline temporary such as
    `epilogue(add=x * 2)` would otherwise be freed - and its memory reused by
    the caching allocator - before the kernel reads it)."""
    e = L.IgrEpilogue()
    e._refs = (add, acc, row_scale, row_mask, col_mask)
    if row_mask is not None:
        e.row_mask = row_mask.data_ptr()
    if col_mask is not None:
        e.col_mask = col_mask.data_ptr()
    if row_scale is not None:
        _f32(row_scale)
        e.row_scale = row_scale.data_ptr()
    e.alpha, e.beta = alpha, beta
    if add is not None:
        e.add, e.ld_add = add.data_ptr(), add.stride(0)
    if acc is not None:
        e.acc, e.ld_acc = acc.data_ptr(), acc.stride(0)
    e.acc_mode, e.acc_div, e.skip_y = acc_mode, acc_div, int(skip_y)
    return e


def spmm(g: Graph, x, rhs=None, out=None, epi=None):
    """y = A x (gspmm 'mul'/'sum'); rhs = edge weights by edge id (None = 1)."""
    _dev(x, rhs, out)
    x, ldx = _rows(x)
    if x.shape[0] < g.n_cols:
        raise IgrError(f'lhs has {x.shape[0]} rows, graph has {g.n_cols} source nodes')
    d = x.shape[1]
    if rhs is not None:
        _f32(rhs)
        if rhs.numel() != g.nnz:
            raise IgrError(f'rhs has {rhs.numel()} values, graph has {g.nnz} edges')
        rhs = rhs.contiguous()
    if out is None and epi is None and d == 1 and g.nnz and g.n_rows:
        return spmv(g, x[:, 0], rhs).view(-1, 1)  # one value per node: the streamed-CSR kernel
    if out is None and epi is None and d not in _SCHEDULED_WIDTHS and g.nnz and g.n_rows:
        return _spmm_other_width(g, x, rhs, d)
    if out is None:
        out = torch.empty(g.n_rows, d, dtype=torch.float32, device=x.device)
    if out.shape[0] < g.n_rows or out.shape[1] != d or out.stride(1) != 1:
        raise IgrError(f'spmm out {tuple(out.shape)} for {g.n_rows} rows x {d}')
    if out.dtype != torch.float32:
        raise IgrError('spmm out must be float32')
    if g.nnz and g.n_rows:
        ws = g.workspace(d)
        L.call('igr_spmm_f32', ctypes.byref(g.csr), d, _p(x), ldx, _p(rhs), _p(out), out.stride(0),
               None if epi is None else ctypes.byref(epi), _p(ws), _stream())
    elif epi is None or (epi.acc_mode == 0 and not epi.add):
        out.zero_()
    else:
        L.call('igr_spmm_f32', ctypes.byref(g.csr), d, _p(x), ldx, _p(rhs), _p(out), out.stride(0),
               ctypes.byref(epi), None, _stream())
    return out


def spmv(g: Graph, x, rhs=None):
    """y[r] = sum_{p in row r} rhs[eid(p)] x[col[p]]: one value per node (igr_spmv_f32), the
    width-1 gspmm 'mul'/'sum'.  No gradient."""
    _dev(x, rhs)
    x = _f32(x).contiguous().view(-1)
    if x.numel() < g.n_cols:
        raise IgrError(f'spmv: x has {x.numel()} values, graph has {g.n_cols} source nodes')
    if rhs is not None:
        rhs = _f32(rhs).contiguous()
        if rhs.numel() != g.nnz:
            raise IgrError(f'rhs has {rhs.numel()} values, graph has {g.nnz} edges')
    y = torch.empty(g.n_rows, dtype=torch.float32, device=x.device)
    L.call('igr_spmv_f32', ctypes.byref(g.csr), _p(x), _p(rhs), _p(y), _stream())
    return y


# Widths the scheduled SpMM kernel is built for.  Any other width goes through it too, in
# column blocks of these widths with the last one zero-padded: the any-width kernel of the
# library gives a row to one wave and a feature to one lane, so a hub row at width 1 is one
# lane's loop (712 us against 20 us on a MovieLens-1M-shaped graph).  Same sums, column by column.
_SCHEDULED_WIDTHS = (32, 64, 128, 256)


def _spmm_other_width(g, x, rhs, d):
    out = torch.empty(g.n_rows, d, dtype=torch.float32, device=x.device)
    c = 0
    while c < d:
        left = d - c
        w = 256 if left >= 256 else next(v for v in _SCHEDULED_WIDTHS if v >= left)
        n = min(w, left)
        if n == w and c % 4 == 0 and x.stride(0) % 4 == 0 and d % 4 == 0:
            spmm(g, x[:, c:c + w], rhs, out=out[:, c:c + w])  # a column block in place (16-byte aligned views)
        else:
            xp = torch.zeros(x.shape[0], w, dtype=torch.float32, device=x.device)
            xp[:, :n] = x[:, c:c + n]
            out[:, c:c + n] = spmm(g, xp, rhs)[:, :n]
        c += n
    return out


def spmm_heads(g: Graph, x, rhs, h, out=None):
    """Per-head SpMM (igr_spmm_heads_f32): out[:, j*d:(j+1)*d] = A_{rhs[:, j]} x[:, j*d:(j+1)*d],
    rhs [nnz, h] by edge id - the h-head SDDMM's backward without per-head copies of rhs."""
    _dev(x, rhs, out)
    x, ldx = _rows(x)
    if x.shape[0] < g.n_cols or x.shape[1] % h:
        raise IgrError(f'spmm_heads: lhs {tuple(x.shape)} for {g.n_cols} source nodes, h={h}')
    d = x.shape[1] // h
    rhs = _f32(rhs).contiguous()
    if rhs.numel() != g.nnz * h:
        raise IgrError(f'spmm_heads: rhs has {rhs.numel()} values, graph has {g.nnz} edges x {h} heads')
    if out is None:
        out = torch.empty(g.n_rows, h * d, dtype=torch.float32, device=x.device)
    if out.shape[0] < g.n_rows or out.shape[1] != h * d or out.stride(1) != 1 or out.dtype != torch.float32:
        raise IgrError(f'spmm_heads out {tuple(out.shape)} for {g.n_rows} rows x {h * d}')
    if g.n_rows:
        L.call('igr_spmm_heads_f32', ctypes.byref(g.csr), h, d, _p(x), ldx, _p(rhs), _p(out), out.stride(0),
               _p(g.workspace(d)), _stream())
    return out


class ScaledWeights:
    """Edge weights w = row_scale[r] * col_scale[c], dropout fused in-kernel with
    keep probability `keep` and a counter-based mask keyed by (seed, offset,
    the edge's (row, column) in the frame it was drawn for) -
    igr_spmm_scaled_f32.  For a graph whose values are row-constant (the IGCN
    feature graph) this replaces the per-edge value array, the rand tensor and
    the dropout pass.  `swap`: applied to the reverse of that frame."""

    def __init__(self, row_scale=None, col_scale=None, keep=1.0, seed=0, offset=0, swap=False, offset_dev=None):
        self.row_scale, self.col_scale = row_scale, col_scale
        self.keep, self.seed, self.offset = float(keep), int(seed), int(offset)
        self.swap = bool(swap)
        self.offset_dev = offset_dev  # device int64 counter added to offset (hipGraph-captured steps)

    def transposed(self):
        return ScaledWeights(self.col_scale, self.row_scale, self.keep, self.seed, self.offset, not self.swap,
                             self.offset_dev)


def spmm_scaled(g: Graph, x, w: ScaledWeights, out=None, epi=None):
    """y = A_w x with ScaledWeights w (see igr_spmm_scaled_f32)."""
    _dev(x, w.row_scale, w.col_scale, out)
    x, ldx = _rows(x)
    if x.shape[0] < g.n_cols:
        raise IgrError(f'lhs has {x.shape[0]} rows, graph has {g.n_cols} source nodes')
    if w.row_scale is not None and w.row_scale.numel() != g.n_rows:
        raise IgrError('row_scale must have n_rows entries')
    if w.col_scale is not None and w.col_scale.numel() != g.n_cols:
        raise IgrError('col_scale must have n_cols entries')
    d = x.shape[1]
    if out is None:
        out = torch.empty(g.n_rows, d, dtype=torch.float32, device=x.device)
    L.call('igr_spmm_scaled_f32', ctypes.byref(g.csr), d, _p(x), ldx, _p(w.row_scale), _p(w.col_scale), w.keep,
           ctypes.c_uint64(w.seed & (2 ** 64 - 1)), ctypes.c_uint64(w.offset & (2 ** 64 - 1)), _p(w.offset_dev),
           int(w.swap), _p(out),
           out.stride(0), None if epi is None else ctypes.byref(epi), _p(g.workspace(d)), _stream())
    return out


def dropout_uniforms(g: Graph, seed, offset, swap=False, offset_dev=None):
    """The uniforms ScaledWeights(seed, offset, swap, offset_dev)'s dropout draws on g, per CSR position."""
    out = torch.empty(g.nnz, dtype=torch.float32, device=g.device)
    L.call('igr_dropout_uniforms', ctypes.byref(g.csr), ctypes.c_uint64(seed & (2 ** 64 - 1)),
           ctypes.c_uint64(offset & (2 ** 64 - 1)), _p(offset_dev), int(bool(swap)), _p(out), _stream())
    return out


def feat_row_values(row_sum, exponent, out=None):
    """Per-row row_sum ** exponent (IGCN.update_feat_mat's value, model.py:4127-4130)."""
    fresh = out is None
    _dev(row_sum, out)
    out = torch.empty_like(row_sum) if out is None else out
    if out.numel() != row_sum.numel() or out.dtype != torch.float32 or not out.is_contiguous():
        raise IgrError(f'feat_row_values: out has {out.numel()} values for {row_sum.numel()} rows')
    L.call('igr_feat_values_f32', row_sum.numel(), None, _p(row_sum), float(exponent), _p(out), _stream())
    return _written(out, fresh)


def _feat_spmm(feat, x, fw, out=None, epi=None, reverse=False):
    """Feature-graph SpMM with per-edge values (tensor) or ScaledWeights."""
    g = feat.reverse() if reverse else feat
    if isinstance(fw, ScaledWeights):
        return spmm_scaled(g, x, fw.transposed() if reverse else fw, out=out, epi=epi)
    return spmm(g, x, fw, out=out, epi=epi)


def _prescale(fw):
    """Row scale to fold into dx_0 before the transposed feature SpMM (None
    unless fw is ScaledWeights with a row scale only): F^T diag(s) M dx =
    F^T M (s * dx), so the reverse SpMM draws the mask but gathers no per-edge
    column scale."""
    if isinstance(fw, ScaledWeights) and fw.row_scale is not None and fw.col_scale is None:
        return fw.row_scale
    return None


def _feat_spmm_rev(feat, dx, fw, prescaled, epi=None):
    """demb = F_w^T dx; `prescaled` means dx already carries fw's row scale."""
    if prescaled:
        return spmm_scaled(feat.reverse(), dx, ScaledWeights(None, None, fw.keep, fw.seed, fw.offset, not fw.swap,
                                                             fw.offset_dev), epi=epi)
    return _feat_spmm(feat, dx, fw, reverse=True, epi=epi)


def neighbor_mask(adj, rows):
    """Bitmap of `rows` and all their neighbours in the square graph adj
    (igr_rowset_mark_neighbors): where a batch's last layer reads the layer below."""
    mask = torch.zeros((adj.n_rows + 31) // 32, dtype=torch.int32, device=rows.device)
    L.call('igr_rowset_mark_neighbors', ctypes.byref(adj.csr), rows.numel(), _p(rows), _p(mask), 1,
           _p(_mark_scratch(adj)), _stream())
    return mask


def _mark_scratch(g):
    """Per-graph uint8[n_cols] byte map for igr_rowset_mark_neighbors (zero between uses)."""
    s = getattr(g, '_mark_bytes', None)
    if s is None:
        s = torch.zeros(max(g.n_cols, 1) + 16, dtype=torch.uint8, device=g.device)
        g._mark_bytes = s
    return s


def column_mask(g, rows, extra=None, out=None):
    """Bitmap over g's columns: the columns of `rows` (int64, may be empty), plus
    the column ids in `extra` (int64 or None)."""
    if out is None:
        out = torch.zeros((g.n_cols + 31) // 32, dtype=torch.int32, device=g.device)
    if rows is not None and rows.numel():
        rows = rows.to(torch.int64).contiguous()
        L.call('igr_rowset_mark_neighbors', ctypes.byref(g.csr), rows.numel(), _p(rows), _p(out), 0,
               _p(_mark_scratch(g)), _stream())
    if extra is not None and extra.numel():
        extra = extra.to(torch.int64).contiguous()
        L.call('igr_bitmap_set', extra.numel(), _p(extra), _p(out), _stream())
    return out


def sddmm_dot(g: Graph, u, v, h=1, out=None):
    """out[eid, j] = <u[row, j, :], v[col, j, :]>; u: [n_rows, h*d], v: [n_cols, h*d]."""
    _dev(u, v, out)
    u, ldu = _rows(u.reshape(u.shape[0], -1))
    v, ldv = _rows(v.reshape(v.shape[0], -1))
    d = u.shape[1] // h
    if u.shape[0] < g.n_rows or v.shape[0] < g.n_cols or u.shape[1] != v.shape[1] or d * h != u.shape[1]:
        raise IgrError(f'sddmm shapes: u {tuple(u.shape)}, v {tuple(v.shape)}, h={h} for graph '
                       f'{g.n_rows}x{g.n_cols}')
    if out is None:
        out = torch.empty(g.nnz, h, dtype=torch.float32, device=u.device)
    L.call('igr_sddmm_dot_f32', ctypes.byref(g.csr), h, d, _p(u), ldu, _p(v), ldv, _p(out), _stream())
    return out


def sddmm_shared(g: Graph, u, v, h, out=None):
    """out[eid, j] = <u[row, j, :], v[col, :]>: one source row of d floats serves all h heads
    (igr_sddmm_shared_f32); u: [n_rows, h*d], v: [n_cols, d]."""
    _dev(u, v, out)
    u, ldu = _rows(u.reshape(u.shape[0], -1))
    v, ldv = _rows(v)
    d = v.shape[1]
    if u.shape[0] < g.n_rows or v.shape[0] < g.n_cols or u.shape[1] != h * d:
        raise IgrError(f'sddmm_shared shapes: u {tuple(u.shape)}, v {tuple(v.shape)}, h={h} for graph '
                       f'{g.n_rows}x{g.n_cols}')
    if out is None:
        out = torch.empty(g.nnz, h, dtype=torch.float32, device=u.device)
    L.call('igr_sddmm_shared_f32', ctypes.byref(g.csr), h, d, _p(u), ldu, _p(v), ldv, _p(out), _stream())
    return out


def spmm_shared_heads(g: Graph, x, rhs, h, out=None):
    """out[r, j*d:(j+1)*d] = sum_{p in row r} rhs[eid(p), j] * x[col_p, :] (igr_spmm_shared_heads_ws_f32)."""
    _dev(x, rhs, out)
    x, ldx = _rows(x)
    d = x.shape[1]
    rhs = _f32(rhs).contiguous()
    if x.shape[0] < g.n_cols or rhs.numel() != g.nnz * h:
        raise IgrError(f'spmm_shared_heads: x {tuple(x.shape)}, rhs {tuple(rhs.shape)} for {g.nnz} edges x {h} heads')
    if out is None:
        out = torch.empty(g.n_rows, h * d, dtype=torch.float32, device=x.device)
    ws = g.workspace(h * d)  # chunk partials of the split rows (None when no row is split)
    L.call('igr_spmm_shared_heads_ws_f32', ctypes.byref(g.csr), h, d, _p(x), ldx, _p(rhs), _p(out), out.stride(0),
           _p(ws), 0 if ws is None else ws.numel() * 4, _stream())
    return out


def segment_reduce(g: Graph, x, reduce='sum'):
    _dev(x)
    x = _f32(x).contiguous()
    h = 1 if x.dim() == 1 else x.shape[1]
    if x.shape[0] != g.nnz:
        raise IgrError(f'segment_reduce: {x.shape[0]} edge values for {g.nnz} edges')
    out = torch.empty(g.n_rows, h, dtype=torch.float32, device=x.device)
    L.call('igr_segment_reduce_f32', ctypes.byref(g.csr), h, _p(x), 1 if reduce == 'max' else 0, _p(out),
           _stream())
    return out if x.dim() > 1 else out[:, 0]


# Rows beyond this many edges make the edge softmax go chunk by chunk over the split rows
# (three launches, any row length spread over the chip); below it a workgroup per split row
# is as fast or faster (MovieLens-1M-shaped feature graph, longest row 4,124 edges: 38 + 37 us
# against 39 + 43 us forward + backward; a 2 M-edge row: 10.7 ms against 0.5 ms).
SOFTMAX_CHUNKED_ROW_EDGES = 8192


def _softmax_workspace(g, h):
    """Per-chunk max / sum slots for the chunked edge softmax, or None (no very long row)."""
    return g.workspace(2 * h) if g.max_row_edges > SOFTMAX_CHUNKED_ROW_EDGES else None


def att_softmax(g: Graph, alpha, sqrt_d, keep=None):
    """keep: optional [nnz] edge values; edges with keep == 0 are absent (dropped)."""
    _dev(alpha, keep)
    alpha = _f32(alpha).contiguous()
    h = alpha.shape[1]
    if alpha.shape[0] != g.nnz:
        raise IgrError(f'att_softmax: {alpha.shape[0]} edge rows for {g.nnz} edges')
    w = torch.empty(g.nnz, dtype=torch.float32, device=alpha.device)
    rmax = torch.empty(g.n_rows, h, dtype=torch.float32, device=alpha.device)
    rsum = torch.empty_like(rmax)
    keep = None if keep is None else keep.contiguous()
    ws = _softmax_workspace(g, h)
    L.call('igr_att_softmax_ws_f32', ctypes.byref(g.csr), h, _p(alpha), _p(keep), float(sqrt_d), _p(w), _p(rmax),
           _p(rsum), _p(ws), 0 if ws is None else ws.numel() * 4, _stream())
    return w, rmax, rsum


def att_softmax_bwd(g: Graph, alpha, sqrt_d, rmax, rsum, dw, keep=None):
    _dev(alpha, dw, keep)
    dalpha = torch.empty_like(alpha)
    keep = None if keep is None else keep.contiguous()
    ws = _softmax_workspace(g, alpha.shape[1])
    L.call('igr_att_softmax_bwd_ws_f32', ctypes.byref(g.csr), alpha.shape[1], _p(alpha), _p(keep), float(sqrt_d),
           _p(rmax), _p(rsum), _p(dw.contiguous()), _p(dalpha), _p(ws), 0 if ws is None else ws.numel() * 4, _stream())
    return dalpha


def edge_dropout_counter(g: Graph, val, p, seed, offset, swap=False, offset_dev=None, out=None):
    """edge_dropout(val, dropout_uniforms(g, seed, offset, ...), p) in one pass, no rand array
    (igr_edge_dropout_counter_f32); val and out by edge id."""
    fresh = out is None
    _dev(val, out, offset_dev)
    val = _f32(val).contiguous()
    if val.numel() != g.nnz:
        raise IgrError(f'edge_dropout_counter: {val.numel()} values for {g.nnz} edges')
    if out is None:
        out = torch.empty_like(val)
    L.call('igr_edge_dropout_counter_f32', ctypes.byref(g.csr), _p(val), float(p), ctypes.c_uint64(seed & (2 ** 64 - 1)),
           ctypes.c_uint64(offset & (2 ** 64 - 1)), _p(offset_dev), int(swap), _p(out), _stream())
    return _written(out, fresh)


def edge_dropout(val, rand, p, out=None):
    fresh = out is None
    _dev(val, rand, out)
    if rand.numel() != val.numel():
        raise IgrError('edge_dropout: rand and val sizes differ')
    if out is None:
        out = torch.empty_like(val)
    L.call('igr_edge_dropout_f32', val.numel(), _p(val), _p(rand), float(p), _p(out), _stream())
    return _written(out, fresh)


def feat_values(g: Graph, row_sum, exponent, out=None):
    fresh = out is None
    _dev(row_sum, out)
    if row_sum.numel() != g.n_rows:
        raise IgrError('feat_values: row_sum size differs from n_rows')
    if out is None:
        out = torch.empty(g.nnz, dtype=torch.float32, device=row_sum.device)
    if out.numel() != g.nnz or out.dtype != torch.float32 or not out.is_contiguous():
        raise IgrError(f'feat_values: out has {out.numel()} values, the graph has {g.nnz} edges '
                       f'(a buffer cached for another feature graph?)')
    L.call('igr_feat_values_f32', g.n_rows, _p(g.row_ptr), _p(row_sum), float(exponent), _p(out), _stream())
    return _written(out, fresh)


def gather_rows(src, idx, offset=0):
    _dev(src, idx)
    src, lds = _rows(src)
    idx = idx.to(torch.int64).contiguous()
    out = torch.empty(idx.numel(), src.shape[1], dtype=torch.float32, device=src.device)
    L.call('igr_gather_rows_f32', idx.numel(), src.shape[1], _p(idx), int(offset), _p(src), lds, _p(out),
           out.stride(0), _stream())
    return out


def rowsort(idx0, off0=0, idx1=None, off1=0, idx2=None, off2=0):
    """Sorted (row << 32 | entry) keys of the concatenation [idx0 + off0; idx1 + off1;
    idx2 + off2] (igr_rowsort): the order every fixed-order accumulation below
    walks.  Returns an int64 tensor whose first n_total entries are the keys."""
    _dev(idx0, idx1, idx2)
    arrs = [a.to(torch.int64).contiguous() for a in (idx0, idx1, idx2) if a is not None]
    n = arrs[0].numel()
    if any(a.numel() != n for a in arrs):
        raise IgrError('rowsort: index arrays must have the same length')
    size = int(L.lib().igr_rowsort_size(n * len(arrs)))
    keys = torch.empty(max(size, 1), dtype=torch.int64, device=idx0.device)
    keys._refs = arrs
    L.call('igr_rowsort', n, _p(arrs[0]), int(off0), _p(arrs[1]) if len(arrs) > 1 else None, int(off1),
           _p(arrs[2]) if len(arrs) > 2 else None, int(off2), _p(keys), _stream())
    return keys


def scatter_add_rows(dst, idx, src, offset=0, sorted_keys=None):
    """dst[idx[i] + offset] += src[i], each row's terms added for i ascending
    (deterministic; sorted_keys = rowsort(idx, offset) when the caller has it)."""
    _dev(dst, idx, src)
    src, lds = _rows(src)
    if idx.numel() != src.shape[0]:
        raise IgrError(f'scatter_add_rows: {idx.numel()} indices for {src.shape[0]} rows')
    if _f32(dst).stride(1) != 1 or dst.shape[1] != src.shape[1]:
        raise IgrError('scatter_add_rows: dst must be [n, d] float32 with unit inner stride')
    if sorted_keys is None:
        sorted_keys = rowsort(idx, offset)
    L.call('igr_scatter_add_rows_f32', idx.numel(), src.shape[1], _p(sorted_keys), _p(src), lds, _p(dst),
           dst.stride(0), _stream())
    return dst


def _bpr_call(B, d, users, pos, neg, off_u, off_i, t, w, loss, l2, g_loss, g_l2, gl_dev, g2_dev, grad, ld_grad,
              dw, sorted_keys):
    """igr_bpr_fwd_bwd_f32 with its backward workspace."""
    ws = None
    if (grad is not None and sorted_keys is not None) or dw is not None:
        ws = torch.empty(int(L.lib().igr_bpr_workspace_floats(B, d)), dtype=torch.float32, device=t.device)
    L.call('igr_bpr_fwd_bwd_f32', B, d, _p(users), _p(pos), _p(neg), int(off_u), int(off_i), _p(t), t.stride(0),
           _p(w), _p(loss), _p(l2), g_loss, g_l2, _p(gl_dev), _p(g2_dev), _p(grad), ld_grad, _p(dw),
           _p(sorted_keys), _p(ws), _stream())


def mask_scores(scores, row_ptr, cols):
    """scores[r, cols[row_ptr[r]:row_ptr[r+1]]] = -inf in place (row_ptr: int64
    [n_rows + 1], absolute offsets into cols, e.g. a slice of a whole CSR)."""
    _dev(scores, row_ptr, cols)
    _f32(scores)
    if scores.stride(1) != 1:
        raise IgrError('mask_scores: scores need unit inner stride')
    n = scores.shape[0]
    if row_ptr.numel() < n + 1:
        raise IgrError('mask_scores: row_ptr needs n_rows + 1 entries')
    L.call('igr_mask_scores_f32', n, _p(row_ptr), _p(cols), _p(scores), scores.stride(0), _stream())
    return scores


def topk(scores, k, values=True):
    """Per-row top k (value descending, ties by index ascending): (values, indices int64)."""
    _dev(scores)
    _f32(scores)
    if scores.dim() != 2 or scores.stride(1) != 1:
        raise IgrError('topk: 2-D scores with unit inner stride expected')
    n, m = scores.shape
    idx = torch.empty(n, k, dtype=torch.int64, device=scores.device)
    val = torch.empty(n, k, dtype=torch.float32, device=scores.device) if values else None
    L.call('igr_topk_f32', n, m, _p(scores), scores.stride(0), int(k), _p(val), _p(idx), _stream())
    return val, idx


def gemm(a, b, bias=None, trans_a=False, trans_b=False):
    """C = A(m,k) B(k,n) + bias; b is [n, k] (Linear weight) unless trans_b."""
    _dev(a, b, bias)
    a, _ = _rows(a)  # rows may be strided (a column block of a wider matrix)
    b, _ = _rows(b)
    m, k = (a.shape[1], a.shape[0]) if trans_a else a.shape
    n = b.shape[1] if trans_b else b.shape[0]
    kb = b.shape[0] if trans_b else b.shape[1]
    if kb != k:
        raise IgrError(f'gemm inner dims differ: {k} vs {kb}')
    c = torch.empty(m, n, dtype=torch.float32, device=a.device)
    wsb = int(L.lib().igr_gemm_workspace_size(m, n, k))  # split-K workspace (few output tiles, long K)
    ws = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=a.device) if wsb > 0 else None
    L.call('igr_gemm_f32', m, n, k, _p(a), a.stride(0), int(trans_a), _p(b), b.stride(0), int(trans_b),
           _p(None if bias is None else bias.contiguous()), _p(c), c.stride(0), _p(ws), wsb, _stream())
    return c


def linear_wgrad(dy, x, want_db=True):
    """(dW, db) of y = x W^T + b over all rows: dW = dy^T x, db = column sums of dy.  Shapes the
    streamed kernel takes (igr_linear_wgrad_f32) get both from one pass over dy and x; others
    get dW from the split-K GEMM and db = None (the caller sums)."""
    _dev(dy, x)
    dy, x = _f32(dy).contiguous(), _f32(x).contiguous()
    m, n_out = dy.shape
    k_in = x.shape[1]
    if x.shape[0] != m:
        raise IgrError(f'linear_wgrad: dy has {m} rows, x has {x.shape[0]}')
    wsb = int(L.lib().igr_linear_wgrad_workspace_size(m, n_out, k_in))
    if wsb <= 0 or dy.data_ptr() % 16 or x.data_ptr() % 16:
        return gemm(dy, x, trans_a=True, trans_b=True), None
    ws = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=dy.device)
    dw = torch.empty(n_out, k_in, dtype=torch.float32, device=dy.device)
    db = torch.empty(n_out, dtype=torch.float32, device=dy.device) if want_db else None
    L.call('igr_linear_wgrad_f32', m, n_out, k_in, _p(dy), dy.stride(0), _p(x), x.stride(0), _p(dw), k_in, _p(db),
           _p(ws), wsb, _stream())
    return dw, db


# ------------------------------------------------------------------ autograd

class GSpMMSum(torch.autograd.Function):
    """gspmm(g, 'mul', 'sum', x, rhs); backward: dx = A^T dy (reverse graph),
    drhs[e] = <dy[row_e], x[col_e]> (u_dot_v SDDMM)."""

    @staticmethod
    def forward(ctx, g, x, rhs):
        ctx.g = g
        ctx.save_for_backward(x if (rhs is not None and rhs.requires_grad) else None, rhs)
        return spmm(g, x, rhs)

    @staticmethod
    def backward(ctx, dy):
        x, rhs = ctx.saved_tensors
        g = ctx.g
        dx = drhs = None
        dy = dy.contiguous()
        if ctx.needs_input_grad[1]:
            rev = g.reverse()
            if rhs is not None and rev.edge_id is not None and rhs.numel() == rev.nnz:
                # the reverse graph reads the values through its edge ids; a model's layers share one
                # value tensor, so permute it once and let every layer's product stream it in order
                dx = spmm(rev.positional(), dy, _reverse_order_values(rev, rhs))
            else:
                dx = spmm(rev, dy, rhs)
        if ctx.needs_input_grad[2]:
            drhs = sddmm_dot(g, dy, x, 1).view(-1)
        return None, dx, drhs


def _reverse_order_values(rev, vals):
    """vals[rev.edge_id], kept for as long as `vals` itself lives and is the tensor asked about
    (the cache holds a weak reference and the tensor's version: another tensor, or this one
    after an in-place write, is permuted afresh; when the tensor dies the copy is dropped)."""
    hit = rev.__dict__.get('_perm_cache')
    if hit is not None and hit[0]() is vals and hit[1] == vals._version:
        return hit[2]
    perm = vals.detach()[rev.edge_id]

    def forget(ref, rev=rev):  # the value tensor is gone: so is its permuted copy
        held = rev.__dict__.get('_perm_cache')
        if held is not None and held[0] is ref:
            del rev.__dict__['_perm_cache']
    rev._perm_cache = (weakref.ref(vals, forget), vals._version, perm)
    return perm


class GSDDMMDot(torch.autograd.Function):
    """out[e, j] = <u[row_e, j], v[col_e, j]> for h heads; backward are per-head SpMMs."""

    @staticmethod
    def forward(ctx, g, u, v, h):
        ctx.g, ctx.h = g, h
        ctx.save_for_backward(u, v)
        return sddmm_dot(g, u, v, h)

    @staticmethod
    def backward(ctx, dout):
        u, v = ctx.saved_tensors
        g, h = ctx.g, ctx.h
        du = dv = None
        dout = dout.contiguous()
        if ctx.needs_input_grad[1]:
            du = spmm_heads(g, v, dout, h, out=torch.empty_like(u))
        if ctx.needs_input_grad[2]:
            dv = spmm_heads(g.reverse(), u, dout, h, out=torch.empty_like(v))
        return None, du, dv, None


class GSDDMMShared(torch.autograd.Function):
    """out[e, j] = <u[row_e, j], v[col_e]> with v shared by the heads; backward:
    du[r, j] = sum_e dout[e, j] v[col_e] (one gather per edge for all heads).  v takes
    no gradient here (AttIGCN detaches the embedding on this path, model.py:4258)."""

    @staticmethod
    def forward(ctx, g, u, v, h):
        if v.requires_grad:
            raise IgrError('gsddmm_shared: the shared source operand takes no gradient; detach it')
        ctx.g, ctx.h = g, h
        ctx.save_for_backward(v)
        ctx.u_shape = u.shape
        return sddmm_shared(g, u, v, h)

    @staticmethod
    def backward(ctx, dout):
        (v,) = ctx.saved_tensors
        du = None
        if ctx.needs_input_grad[1]:
            du = spmm_shared_heads(ctx.g, v, dout.contiguous(), ctx.h).view(ctx.u_shape)
        return None, du, None, None


class SegmentSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, x):
        ctx.g = g
        return segment_reduce(g, x, 'sum')

    @staticmethod
    def backward(ctx, dout):
        g = ctx.g
        d2 = dout if dout.dim() == 2 else dout[:, None]
        dx = gather_rows(d2.contiguous(), g.edge_rows())
        return None, dx if dout.dim() == 2 else dx[:, 0]


class SegmentMax(torch.autograd.Function):
    """gspmm(g, 'copy_rhs', 'max', None, x) with DGL's backward: each row's gradient goes to
    the edge that holds the row's maximum (the first one in edge order on ties, as a
    compare-greater scan over the row finds it).  The API-compatible path of model.py:4270;
    the fused edge softmax (AttSoftmax) needs no such gradient."""

    @staticmethod
    def forward(ctx, g, x):
        out = segment_reduce(g, x, 'max')
        ctx.g = g
        ctx.save_for_backward(x, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, out = ctx.saved_tensors
        g = ctx.g
        rows = g.edge_rows()
        x2 = x if x.dim() == 2 else x[:, None]
        o2 = out if out.dim() == 2 else out[:, None]
        d2 = dout if dout.dim() == 2 else dout[:, None]
        is_max = x2 == o2[rows]
        nnz = x2.shape[0]
        idx = torch.arange(nnz, device=x.device)[:, None].expand_as(x2)
        cand = torch.where(is_max, idx, torch.full_like(idx, nnz))
        first = torch.full(o2.shape, nnz, dtype=idx.dtype, device=x.device)
        first = first.scatter_reduce(0, rows[:, None].expand_as(x2), cand, 'amin')
        dx = torch.where(cand == first[rows], d2[rows], torch.zeros((), dtype=d2.dtype, device=x.device))
        return None, dx if x.dim() == 2 else dx[:, 0]


class AttSoftmax(torch.autograd.Function):
    """AttIGCN edge softmax + head mean (model.py:4270-4275); `keep` marks the
    edges present after dropout (keep == 0: removed, as dropout_sp_mat does)."""

    @staticmethod
    def forward(ctx, g, alpha, sqrt_d, keep=None):
        w, rmax, rsum = att_softmax(g, alpha, sqrt_d, keep)
        ctx.g, ctx.sqrt_d = g, sqrt_d
        ctx.save_for_backward(alpha, rmax, rsum, keep)
        return w

    @staticmethod
    def backward(ctx, dw):
        alpha, rmax, rsum, keep = ctx.saved_tensors
        return None, att_softmax_bwd(ctx.g, alpha, ctx.sqrt_d, rmax, rsum, dw, keep), None, None


class Linear(torch.autograd.Function):
    """nn.Linear on the MFMA GEMM: y = x W^T + b."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return gemm(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.contiguous()
        dx = gemm(dy, weight, trans_b=True) if ctx.needs_input_grad[0] else None
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        dw = db = None
        if ctx.needs_input_grad[1]:
            dw, db = linear_wgrad(dy, x, want_db)   # one streamed pass gives both when the shape allows
        if want_db and db is None:
            db = dy.sum(0)
        return dx, dw, db


class GatherRows(torch.autograd.Function):
    """rep[idx + offset] with a scatter-add backward."""

    @staticmethod
    def forward(ctx, src, idx, offset):
        ctx.save_for_backward(idx)
        ctx.n, ctx.offset = src.shape[0], offset
        return gather_rows(src, idx, offset)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        dsrc = torch.zeros(ctx.n, dy.shape[1], dtype=dy.dtype, device=dy.device)
        return scatter_add_rows(dsrc, idx, dy, ctx.offset), None, None


def linear(x, layer):
    """Apply an nn.Linear through the MFMA GEMM."""
    return Linear.apply(x, layer.weight, layer.bias)


def gather(src, idx, offset=0):
    return GatherRows.apply(src, idx, int(offset))


class CoefProduct(torch.autograd.Function):
    """coef @ b for per-row coefficients that take no gradient (coef [n, k], k small; b [k, d]):
    the gradient of b is coef^T g, a k x d result reduced over all n rows - the split-K GEMM
    (summed in a fixed order) instead of a one-workgroup library kernel."""

    @staticmethod
    def forward(ctx, coef, b):
        ctx.save_for_backward(coef)
        return gemm(coef, b, trans_b=True)

    @staticmethod
    def backward(ctx, g):
        coef, = ctx.saved_tensors
        return None, gemm(coef, g, trans_a=True, trans_b=True)


def coef_product(coef, b):
    return CoefProduct.apply(coef.detach(), b)


LAYER_TAIL_MAX_WIDTH = 256


class LayerTail(torch.autograd.Function):
    """NGCF's layer tail after the two Linear layers (model.py:4040-4042) in one kernel each way:
    r = dropout(leaky_relu(a + b)), nrm = F.normalize(r, p=2, dim=1); returns (r, nrm)."""

    @staticmethod
    def forward(ctx, a, b, keep, keep_scale, slope):
        _dev(a, b, keep)
        a, lda = _rows(a)
        b, ldb = _rows(b)
        n, d = a.shape
        if b.shape != a.shape or (keep is not None and keep.shape != a.shape):
            raise IgrError(f'layer_tail: a {tuple(a.shape)}, b {tuple(b.shape)}')
        keep = None if keep is None else _f32(keep).contiguous()
        r = torch.empty(n, d, dtype=torch.float32, device=a.device)
        nrm = torch.empty_like(r)
        row_norm = torch.empty(n, dtype=torch.float32, device=a.device)
        L.call('igr_layer_tail_f32', n, d, _p(a), lda, _p(b), ldb, _p(keep), float(keep_scale), float(slope), _p(r),
               _p(nrm), d, _p(row_norm), _stream())
        ctx.save_for_backward(r, row_norm, keep)
        ctx.consts = (float(keep_scale), float(slope))
        ctx.set_materialize_grads(False)
        return r, nrm

    @staticmethod
    def backward(ctx, g_r, g_n):
        r, row_norm, keep = ctx.saved_tensors
        n, d = r.shape
        if g_r is None and g_n is None:
            return None, None, None, None, None
        ldr = ldn = 0
        if g_r is not None:
            g_r, ldr = _rows(g_r)
        if g_n is not None:
            g_n, ldn = _rows(g_n)
        dz = torch.empty_like(r)
        L.call('igr_layer_tail_bwd_f32', n, d, _p(g_n), ldn, _p(g_r), ldr, _p(r), _p(row_norm), _p(keep),
               ctx.consts[0], ctx.consts[1], _p(dz), _stream())
        return dz, dz, None, None, None


def layer_tail(a, b, p=0.0, training=False, slope=0.2):
    """(r, F.normalize(r)) with r = F.dropout(F.leaky_relu(a + b, slope), p, training)
    (model.py:4040-4042).  The dropout mask is one Bernoulli(1 - p) draw per element from
    torch's generator of the device."""
    keep, scale = None, 1.0
    if training and p >= 1:  # F.dropout(p=1): all zeros
        keep, scale = torch.zeros(a.shape, dtype=torch.float32, device=a.device), 0.0
    elif training and p > 0:
        keep = torch.empty(a.shape, dtype=torch.float32, device=a.device).bernoulli_(1.0 - p)
        scale = 1.0 / (1.0 - p)
    return LayerTail.apply(a, b, keep, scale, slope)


class Propagate(torch.autograd.Function):
    """rep = mean_l(x_l), x_{l+1} = A x_l, x_0 = F emb (inductive) or emb.

    One fused pass per layer: each SpMM's epilogue accumulates the running
    layer sum, the last one divides by L+1 (model.py:4188-4200, 100-110).
    Backward (A symmetric => A^T = A bit-exactly for D^-1/2 A D^-1/2):
        dx_L = g/(L+1);  dx_l = A^T dx_{l+1} + g/(L+1);  demb = F^T dx_0;
        dfvals[e] = <dx_0[row_e], emb[col_e]> when the feature values need a
        gradient (AttIGCN's attention weights).
    """

    @staticmethod
    def forward(ctx, adj, adj_vals, feat, emb, fvals, n_layers):
        ctx.adj, ctx.feat, ctx.L = adj, feat, n_layers
        scaled = isinstance(fvals, ScaledWeights)
        ctx.fw = fvals if scaled else None
        ctx.save_for_backward(adj_vals, None if scaled else fvals)
        L1 = n_layers + 1
        dev = emb.device
        ctx.emb = emb if (not scaled and fvals is not None and fvals.requires_grad) else None
        if feat is not None:
            x = torch.empty(feat.n_rows, emb.shape[1], dtype=torch.float32, device=dev)
            if n_layers == 0:
                return _feat_spmm(feat, emb, fvals, out=x)
            acc = torch.empty_like(x)
            _feat_spmm(feat, emb, fvals, out=x, epi=epilogue(acc=acc, acc_mode=1))
            own_x = True
        else:
            x = emb.contiguous()
            if n_layers == 0:
                return x.clone()
            acc = x.clone()
            own_x = False  # never write into the caller's embedding table
        y = torch.empty_like(acc)
        for layer in range(n_layers):
            last = layer == n_layers - 1
            spmm(adj, x, adj_vals, out=y, epi=epilogue(acc=acc, acc_mode=2, acc_div=float(L1) if last else 1.0,
                                                   skip_y=last))
            if not last:
                x, y = y, (x if own_x else torch.empty_like(acc))
                own_x = True
        return acc

    @staticmethod
    def backward(ctx, g):
        adj_vals, fvals = ctx.saved_tensors
        if ctx.fw is not None:
            fvals = ctx.fw
        adj, feat, n_layers = ctx.adj, ctx.feat, ctx.L
        L1 = float(n_layers + 1)
        g = g.contiguous()
        rs = _prescale(fvals) if (feat is not None and ctx.needs_input_grad[3]) else None
        if n_layers == 0:
            dx = g if rs is None else g * rs[:, None]
        else:
            dx = g / L1
            at = adj.reverse()
            nxt = torch.empty_like(dx)
            for layer in range(n_layers):
                last = layer == n_layers - 1
                spmm(at, dx, adj_vals, out=nxt, epi=epilogue(beta=1.0 / L1, add=g, row_scale=rs if last else None))
                dx, nxt = nxt, dx
        if feat is None:
            return None, None, None, dx, None, None
        demb = _feat_spmm_rev(feat, dx, fvals, rs is not None) if ctx.needs_input_grad[3] else None
        dfv = None
        if ctx.emb is not None and ctx.needs_input_grad[4]:
            dfv = sddmm_dot(feat, dx, ctx.emb, 1).view(-1)
        return None, None, None, demb, dfv, None


def spmm_rows(g: Graph, x, rows, rhs=None, add_g=None, add_i=None, scale=1.0, out=None):
    """out[i] = scale * ((A x)[rows[i]] + add_g[rows[i]] + add_i[i]) (igr_spmm_rows_f32)."""
    _dev(x, rows, rhs, add_g, add_i, out)
    if g.edge_id is not None and rhs is not None:
        raise IgrError('spmm_rows: rhs by edge id needs a graph without an edge_id permutation')
    x, ldx = _rows(x)
    d = x.shape[1]
    rows = rows.to(torch.int64).contiguous()
    if out is None:
        out = torch.empty(rows.numel(), d, dtype=torch.float32, device=x.device)
    ag, lg = _rows(add_g) if add_g is not None else (None, 0)
    ai, li = _rows(add_i) if add_i is not None else (None, 0)
    L.call('igr_spmm_rows_f32', ctypes.byref(g.csr), d, _p(rows), rows.numel(), _p(x), ldx,
           _p(None if rhs is None else _f32(rhs).contiguous()), _p(ag), lg, _p(ai), li, float(scale), _p(out),
           out.stride(0), _stream())
    return out


def spmm_push(g: Graph, rows, src, dst, rhs=None, scale=1.0, self_add=False):
    """dst[col[p]] += scale * rhs[p] * src[i] for p in row rows[i] (+ dst[rows[i]] += scale * src[i])."""
    _dev(src, rows, rhs, dst)
    if g.edge_id is not None and rhs is not None:
        raise IgrError('spmm_push: rhs by edge id needs a graph without an edge_id permutation')
    src, lds = _rows(src)
    rows = rows.to(torch.int64).contiguous()
    if dst.stride(1) != 1 or dst.shape[1] != src.shape[1] or dst.shape[0] < g.n_cols:
        raise IgrError('spmm_push: dst must be [n_cols, d] with unit inner stride')
    L.call('igr_spmm_push_f32', ctypes.byref(g.csr), src.shape[1], _p(rows), rows.numel(), _p(src), lds,
           _p(None if rhs is None else _f32(rhs).contiguous()), float(scale), int(bool(self_add)), _p(dst),
           dst.stride(0), _stream())
    return dst


def _rowset(g: Graph):
    """Per-graph bitmap + 64 KB LDS filter (both zero between uses) + slot map over the column space."""
    rs = getattr(g, '_rowset', None)
    if rs is None:
        n = g.n_cols
        rs = (torch.zeros((n + 31) // 32, dtype=torch.int32, device=g.device),
              torch.zeros(1 << 14, dtype=torch.int32, device=g.device),
              torch.empty(max(n, 1), dtype=torch.int32, device=g.device))
        g._rowset = rs
    return rs


def spmm_pull(g: Graph, rows, src, rhs=None, scale=1.0, self_add=False, out=None, row_mask=None, sorted_keys=None):
    """out[c] = scale * (sum_{p in row c} rhs[p] S[col[p]] + self_add S[c]) with
    S[r] = sum of src[i] over rows[i] == r (i ascending) - the atomic-free
    equivalent of spmm_push on the reverse graph (igr_spmm_pull_marked_f32).
    row_mask (a bitmap over the rows): only the marked rows are computed; the
    others of `out` are left as they were.  sorted_keys = rowsort(rows)."""
    _dev(src, rows, rhs, out, row_mask)
    if g.edge_id is not None and rhs is not None:
        raise IgrError('spmm_pull: rhs by edge id needs a graph without an edge_id permutation')
    src, lds = _rows(src)
    d = src.shape[1]
    rows = rows.to(torch.int64).contiguous()
    bits, filt, slot = _rowset(g)
    agg = torch.empty(max(rows.numel(), 1), d, dtype=torch.float32, device=src.device)
    if out is None:
        out = torch.empty(g.n_rows, d, dtype=torch.float32, device=src.device)
    if sorted_keys is None:
        sorted_keys = rowsort(rows)
    st = _stream()
    L.call('igr_rowset_mark', rows.numel(), _p(rows), _p(bits), _p(filt), st)
    L.call('igr_rowset_sum_f32', rows.numel(), d, _p(sorted_keys), _p(src), lds, 1.0, _p(slot), _p(agg),
           agg.stride(0), st)
    L.call('igr_spmm_pull_marked_f32', ctypes.byref(g.csr), d, _p(bits), _p(filt), _p(slot), _p(agg), agg.stride(0),
           _p(None if rhs is None else _f32(rhs).contiguous()), float(scale), int(bool(self_add)), _p(row_mask),
           _p(out), out.stride(0), st)
    L.call('igr_rowset_clear', rows.numel(), _p(rows), _p(bits), _p(filt), st)
    return out


class PropagateRows(torch.autograd.Function):
    """rep[rows] for Propagate's rep, computing the LAST layer only at `rows`.

    Forward: x_0 .. x_{L-1} in full (no running-sum epilogue: the layer mean
    is needed only at the rows), then one workgroup per selected row:
        rep_b = ((A x_{L-1})[rows] + x_{L-1}[rows] + sum_{l<L-1} x_l[rows]) / (L+1).
    Backward (g_b = d loss / d rep_b):
        dx_{L-1} = A^T G + G, G = scatter(g_b/(L+1))   (masked pull; push if A not symmetric)
        dx_l     = A^T dx_{l+1} + scatter(g_b/(L+1))            (full SpMM)
        demb     = F^T dx_0
    Two full-graph SpMMs fewer per training step than rep = Propagate(...)
    followed by a gather; worth it when the batch rows touch far fewer edges
    than the graph has (see model.batch_rep_pays).

    One level further (symmetric adj): the last layer reads x_{L-1} only at
    R = rows + their neighbours, so x_{L-1} (x_0 when L = 1) is computed only
    at R (row_mask), and dx_{L-1} - which is zero off R - is pulled only from
    R (col_mask) in the first full reverse layer.  Exact: skipped terms are
    exact zeros."""

    @staticmethod
    def forward(ctx, adj, adj_vals, feat, emb, fvals, n_layers, rows, aux=None, w=None):
        ctx.adj, ctx.feat, ctx.L = adj, feat, n_layers
        ctx.aux = aux
        scaled = isinstance(fvals, ScaledWeights)
        ctx.fw = fvals if scaled else None
        ctx.save_for_backward(adj_vals, None if scaled else fvals, rows, emb if aux is not None else None, w)
        ctx.emb = emb if (not scaled and fvals is not None and fvals.requires_grad) else None
        L1 = n_layers + 1
        aux_loss = None
        if aux is not None:
            au, ap, an, off = aux
            loss = torch.empty(au.numel(), dtype=torch.float32, device=emb.device)
            _bpr_call(au.numel(), emb.shape[1], au, ap, an, 0, int(off), emb, w, loss, None, 0.0, 0.0, None, None,
                      None, 0, None, None)
            aux_loss = loss.mean()
        mask = neighbor_mask(adj, rows) if (adj.reverse() is adj and adj.n_rows == adj.n_cols) else None
        ctx.mask = mask
        em = None if mask is None else epilogue(row_mask=mask)
        if feat is not None:
            x = _feat_spmm(feat, emb, fvals, epi=em if n_layers == 1 else None)
        else:
            x = emb.contiguous()
        s = None
        for layer in range(n_layers - 1):
            xr = gather_rows(x, rows)
            s = xr if s is None else s.add_(xr)
            x = spmm(adj, x, adj_vals, epi=em if layer == n_layers - 2 else None)
        rep_b = spmm_rows(adj, x, rows, adj_vals, add_g=x, add_i=s, scale=1.0 / L1)
        return rep_b if aux is None else (rep_b, aux_loss)

    @staticmethod
    def backward(ctx, gb, g_aux=None):
        adj_vals, fvals, rows, emb, w = ctx.saved_tensors
        if ctx.fw is not None:
            fvals = ctx.fw
        adj, feat, n_layers = ctx.adj, ctx.feat, ctx.L
        gs = gb.contiguous() / float(n_layers + 1)
        rs = _prescale(fvals) if feat is not None else None
        mask = ctx.mask
        keys = rowsort(rows)  # one sort serves the pull and every scatter of this backward
        if adj.reverse() is adj:
            # with L > 1, dx_{L-1} is read only through the first reverse layer's
            # column mask (the neighbour set R): rows off R are not computed
            dx = spmm_pull(adj, rows, gs, adj_vals, self_add=True, row_mask=mask if n_layers > 1 else None,
                           sorted_keys=keys)
        else:
            dx = torch.zeros(adj.n_cols, gs.shape[1], dtype=torch.float32, device=gs.device)
            spmm_push(adj, rows, gs, dx, adj_vals, self_add=True)
        if n_layers > 1:
            at = adj.reverse()
            nxt = torch.empty_like(dx)
            for layer in range(n_layers - 1):
                last = layer == n_layers - 2
                cm = mask if layer == 0 else None  # dx_{L-1} is zero off the neighbour set
                epi = None
                if (last and rs is not None) or cm is not None:
                    epi = epilogue(row_scale=rs if last else None, col_mask=cm)
                spmm(at, dx, adj_vals, out=nxt, epi=epi)
                scatter_add_rows(nxt, rows, gs if not (last and rs is not None) else gs * rs[rows][:, None],
                                 sorted_keys=keys)
                dx, nxt = nxt, dx
        elif rs is not None:
            dx.mul_(rs[:, None])
        dfv = None
        if feat is None:
            demb = dx
        else:
            cm = mask if n_layers == 1 else None
            demb = _feat_spmm_rev(feat, dx, fvals, rs is not None, epi=None if cm is None else epilogue(col_mask=cm))
            if ctx.emb is not None and ctx.needs_input_grad[4]:
                dfv = sddmm_dot(feat, dx, ctx.emb, 1).view(-1)
        dw = None
        if ctx.aux is not None and g_aux is not None:
            # the aux BPR term's gradient goes straight into demb (no second
            # full-size gradient for autograd to add)
            au, ap, an, off = ctx.aux
            dw = torch.zeros_like(w) if (w is not None and ctx.needs_input_grad[8]) else None
            g_aux = _f32(g_aux).contiguous()
            _bpr_call(au.numel(), emb.shape[1], au, ap, an, 0, int(off), emb, w, None, None, 1.0 / au.numel(), 0.0,
                      g_aux, None, demb, demb.stride(0), dw, rowsort(au, 0, ap, int(off), an, int(off)))
        return None, None, None, demb, dfv, None, None, None, dw


def propagate_rows(adj, emb, n_layers, rows, feat=None, fvals=None, adj_vals=None, aux=None, w=None):
    """propagate(...)[rows] with the last layer computed only at `rows` (repeats allowed).

    aux = (users, pos, neg, off_i): also return the mean aux BPR loss on the
    raw table emb with feature weights w (IGCNTrainer's aux term,
    trainer.py:542-549); its gradient is accumulated into emb's gradient
    inside the backward."""
    if n_layers == 0:
        raise IgrError('propagate_rows needs n_layers >= 1')
    if aux is not None:
        aux = tuple(a.to(torch.int64).contiguous() for a in aux[:3]) + (int(aux[3]),)
        _dev(*aux[:3], w)
    return PropagateRows.apply(adj, adj_vals, feat, emb, fvals, n_layers, rows.to(torch.int64).contiguous(), aux, w)


_ARANGE = {}


def batch_positions(B, device):
    """(arange(B), B + arange(B), 2B + arange(B)) on `device`, cached."""
    key = (B, torch.device(device))
    if key not in _ARANGE:
        a = torch.arange(3 * B, dtype=torch.int64, device=device)
        _ARANGE[key] = (a[:B], a[B:2 * B], a[2 * B:])
    return _ARANGE[key]


def batch_rows(users, pos, neg, n_users):
    """Rows of rep a BPR batch reads, and the positions of (users, pos, neg) in
    them: rows = [users, n_users + pos, n_users + neg] (repeats kept - no
    host sync for a unique())."""
    rows = torch.cat([users.to(torch.int64), pos.to(torch.int64) + n_users, neg.to(torch.int64) + n_users])
    return rows, batch_positions(users.numel(), users.device)


def propagate(adj, emb, n_layers, feat=None, fvals=None, adj_vals=None):
    """Fused get_rep: mean over [x0, A x0, ..., A^L x0], x0 = F emb (feat given) or emb.
    fvals: per-edge feature values (tensor, by edge id) or ScaledWeights."""
    return Propagate.apply(adj, adj_vals, feat, emb, fvals, n_layers)


class BPRLoss(torch.autograd.Function):
    """Fused BPR term: mean_b softplus(<u, n*w> - <u, p*w>) and mean_b l2_b,
    rows gathered from one table t (model.py:4046-4052, trainer.py:536-548)."""

    @staticmethod
    def forward(ctx, t, w, users, pos, neg, off_u, off_i, distinct, keys=None):
        _dev(t, users, pos, neg, w)
        t = t.contiguous()
        B = users.numel()
        loss = torch.empty(B, dtype=torch.float32, device=t.device)
        l2 = torch.empty_like(loss)
        _bpr_call(B, t.shape[1], users, pos, neg, off_u, off_i, t, w, loss, l2, 0.0, 0.0, None, None, None, 0, None,
                  None)
        ctx.save_for_backward(t, w, users, pos, neg)
        ctx.off = (int(off_u), int(off_i))
        ctx.distinct = bool(distinct)
        ctx.keys = keys
        m = means(loss, l2)  # both means in one launch, fixed summation order
        return m[0], m[1]

    @staticmethod
    def backward(ctx, g_loss, g_l2):
        t, w, users, pos, neg = ctx.saved_tensors
        B = users.numel()
        # incoming gradients stay on the device (no float() sync): the kernel scales by them
        gl = None if g_loss is None else _f32(g_loss).contiguous()
        g2 = None if g_l2 is None else _f32(g_l2).contiguous()
        grad = torch.zeros_like(t) if ctx.needs_input_grad[0] else None
        dw = torch.zeros_like(w) if (w is not None and ctx.needs_input_grad[1]) else None
        keys = None
        if grad is not None and not ctx.distinct:
            keys = ctx.keys if ctx.keys is not None else rowsort(users, ctx.off[0], pos, ctx.off[1], neg, ctx.off[1])
        _bpr_call(B, t.shape[1], users, pos, neg, ctx.off[0], ctx.off[1], t, w, None, None,
                  0.0 if gl is None else 1.0 / B, 0.0 if g2 is None else 1.0 / B, gl, g2, grad, t.stride(0), dw, keys)
        return grad, dw, None, None, None, None, None, None, None


def means(a, b=None):
    """[mean(a), mean(b)] of per-sample terms in one launch (igr_means_f32)."""
    _dev(a, b)
    a = _f32(a).contiguous()
    b = None if b is None else _f32(b).contiguous()
    out = torch.empty(2 if b is not None else 1, dtype=torch.float32, device=a.device)
    L.call('igr_means_f32', a.numel(), _p(a), _p(b), _p(out), _stream())
    return out


def loss_combine(bpr, l2=None, aux=None, c_l2=0.0, c_aux=0.0, loss_sum=None, weight=1.0):
    """loss = bpr + (c_l2 * l2 + c_aux * aux) as one launch on detached device
    scalars (trainer.py:551-552); loss_sum += loss * weight when given."""
    _dev(bpr, l2, aux, loss_sum)
    out = torch.empty((), dtype=torch.float32, device=bpr.device)
    L.call('igr_loss_combine_f32', _p(bpr.detach()), _p(None if l2 is None else l2.detach()),
           _p(None if aux is None else aux.detach()), float(c_l2), float(c_aux), float(weight), _p(out),
           _p(loss_sum), _stream())
    return out


def bpr_loss(t, users, pos, neg, off_u, off_i, w=None, distinct=False, keys=None):
    """Returns (mean softplus BPR loss, mean squared-norm term).  distinct: the
    caller guarantees that the 3B table rows read are all different (a table of
    gathered batch rows read at batch_positions), so the gradient needs no sort.
    keys: rowsort(users, off_u, pos, off_i, neg, off_i) when the caller already has it
    (the backward then skips its sort)."""
    return BPRLoss.apply(t, w, users.to(torch.int64).contiguous(), pos.to(torch.int64).contiguous(),
                         neg.to(torch.int64).contiguous(), off_u, off_i, distinct, keys)


# ------------------------------------------------------------------ DGL-compatible API

def graph(edges, num_nodes=None, device='cuda'):
    """dgl.graph((src, dst), num_nodes=n): rows = dst, columns = src; every
    edge kept, edge ids = input positions (model.py:104, 4183, 4194)."""
    src, dst = edges
    src = src.detach().cpu().numpy() if isinstance(src, torch.Tensor) else np.asarray(src)
    dst = dst.detach().cpu().numpy() if isinstance(dst, torch.Tensor) else np.asarray(dst)
    if num_nodes is None:
        num_nodes = int(max(src.max(initial=-1), dst.max(initial=-1)) + 1)
    g, _ = Graph.from_coo(dst, src, num_nodes, num_nodes, None, dedup=False, device=device)
    return g


def gspmm(g, op, reduce_op, lhs_data, rhs_data):
    if op == 'mul' and reduce_op == 'sum':
        if rhs_data is not None and rhs_data.dim() != 1:
            raise IgrError('gspmm mul/sum: rhs_data must be one scalar per edge')
        return GSpMMSum.apply(g, lhs_data, rhs_data)
    if op == 'copy_rhs' and reduce_op == 'sum':
        return SegmentSum.apply(g, rhs_data)
    if op == 'copy_rhs' and reduce_op == 'max':
        if rhs_data.requires_grad and torch.is_grad_enabled():
            return SegmentMax.apply(g, rhs_data)
        return segment_reduce(g, rhs_data, 'max')
    raise IgrError(f'gspmm op ({op}, {reduce_op}) not supported')


def gsddmm(g, op, lhs_data, rhs_data, h=1):
    """u_dot_v with lhs on destination rows and rhs on source columns."""
    if op != 'dot':
        raise IgrError(f'gsddmm op {op} not supported')
    return GSDDMMDot.apply(g, lhs_data, rhs_data, h)


def sqrt_scale(d):
    return float(np.float32(math.sqrt(d)))


def spmm_tiled(tg, x, tile_vals, out=None):
    """y = A x over a TiledGraph: first tile writes, later tiles accumulate in place."""
    _dev(x)
    x, ldx = _rows(x)
    d = x.shape[1]
    if out is None:
        out = torch.empty(tg.n_rows, d, dtype=torch.float32, device=x.device)
    for t, (g, v) in enumerate(zip(tg.tiles, tile_vals)):
        xs = x[tg.bounds[t]:tg.bounds[t + 1]]
        spmm(g, xs, v, out=out, epi=None if t == 0 else epilogue(beta=1.0, add=out))
    return out
