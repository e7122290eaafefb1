"""ctypes binding of the igr C ABI (include/igr.h) -> lib/libigr.so.

This is the reference-side binding a maintainer adds next to the DGL call
sites: plain pointers, sizes and a hipStream_t; no torch
types cross the boundary.  Loading fails loudly if the library is missing -
there is no CPU fallback for the device entry points.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('IGR_LIB', os.path.join(_HERE, 'lib', 'libigr.so'))

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p
SPMM_NOALLOC_MAX_FLOATS = 4 << 20  # IGR_SPMM_NOALLOC_MAX_FLOATS (include/igr.h)


class IgrCsr(ctypes.Structure):
    """struct igr_csr (include/igr.h)."""
    _fields_ = [
        ('n_rows', c_i64), ('n_cols', c_i64), ('nnz', c_i64),
        ('row_ptr', c_vp), ('col_idx', c_vp), ('edge_id', c_vp),
        ('n_order', c_i64), ('order', c_vp),
        ('n_split', c_i64), ('split_row', c_vp), ('split_ptr', c_vp),
        ('n_chunks', c_i64), ('chunk_row', c_vp), ('chunk_beg', c_vp),
        ('chunk_edges', c_i64),
    ]


ADAM_MAX_SLOTS = 16


class IgrAdamSlot(ctypes.Structure):          # struct igr_adam_slot
    _fields_ = [('param', c_vp), ('grad', c_vp), ('exp_avg', c_vp), ('exp_avg_sq', c_vp), ('n', c_i64), ('step', c_i64)]


class IgrEpilogue(ctypes.Structure):
    """struct igr_epilogue (include/igr.h)."""
    _fields_ = [
        ('alpha', c_f32), ('beta', c_f32), ('add', c_vp), ('ld_add', c_i64),
        ('acc', c_vp), ('ld_acc', c_i64), ('acc_mode', c_i32), ('acc_div', c_f32),
        ('skip_y', c_i32), ('row_scale', c_vp), ('row_mask', c_vp), ('col_mask', c_vp),
    ]


_P = ctypes.POINTER
# name -> (restype, argtypes); the full exported surface of include/igr.h
SIGNATURES = {
    'igr_last_error': (ctypes.c_char_p, []),
    'igr_version': (ctypes.c_int, []),
    'igr_device_info': (ctypes.c_int, [ctypes.c_int, _P(ctypes.c_int), _P(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]),
    'igr_csr_from_coo': (ctypes.c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp,
                                        _P(c_i64), c_i32]),
    'igr_count_ids': (ctypes.c_int, [c_i64, c_vp, c_i64, c_vp, c_i32]),
    'igr_select_id_range': (ctypes.c_int, [c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, _P(c_i64), c_i32]),
    'igr_csr_transpose': (ctypes.c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32]),
    'igr_csr_row_sums': (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp]),
    'igr_sym_norm_values': (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    'igr_plan_size': (ctypes.c_int, [c_i64, c_vp, c_i64, c_i64, _P(c_i64), _P(c_i64), _P(c_i64)]),
    'igr_plan_fill': (ctypes.c_int, [c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    'igr_spmm_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, _P(IgrEpilogue), c_vp, c_vp]),
    'igr_spmm_noalloc_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, _P(IgrEpilogue), c_vp]),
    'igr_spmm_heads_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp]),
    'igr_spmm_scaled_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_i64, c_vp, c_vp, c_f32, ctypes.c_uint64,
                                           ctypes.c_uint64, c_vp, c_i32, c_vp, c_i64, _P(IgrEpilogue), c_vp, c_vp]),
    'igr_spmm_rows_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                         c_i64, c_f32, c_vp, c_i64, c_vp]),
    'igr_spmm_push_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_f32, c_i32, c_vp,
                                         c_i64, c_vp]),
    'igr_rowsort_size': (c_i64, [c_i64]),
    'igr_rowsort': (ctypes.c_int, [c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    'igr_rowset_mark': (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    'igr_rowset_mark_neighbors': (ctypes.c_int, [_P(IgrCsr), c_i64, c_vp, c_vp, c_i32, c_vp, c_vp]),
    'igr_bitmap_set': (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp]),
    'igr_rowset_sum_f32': (ctypes.c_int, [c_i64, c_i32, c_vp, c_vp, c_i64, c_f32, c_vp, c_vp, c_i64, c_vp]),
    'igr_spmm_pull_marked_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_f32,
                                                c_i32, c_vp, c_vp, c_i64, c_vp]),
    'igr_rowset_clear': (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    'igr_mask_scores_f32': (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_i64, c_vp]),
    'igr_topk_f32': (ctypes.c_int, [c_i64, c_i64, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp]),
    'igr_dropout_uniforms': (ctypes.c_int, [_P(IgrCsr), ctypes.c_uint64, ctypes.c_uint64, c_vp, c_i32, c_vp, c_vp]),
    'igr_edge_dropout_counter_f32': (ctypes.c_int, [_P(IgrCsr), c_vp, c_f32, ctypes.c_uint64, ctypes.c_uint64, c_vp,
                                                    c_i32, c_vp, c_vp]),
    'igr_sddmm_dot_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    'igr_sddmm_shared_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    'igr_spmm_shared_heads_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    'igr_spmm_shared_heads_workspace_size': (c_i64, [_P(IgrCsr), c_i32, c_i32]),
    'igr_spmm_shared_heads_ws_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                                    c_i64, c_vp]),
    'igr_segment_reduce_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_i32, c_vp, c_vp]),
    'igr_att_softmax_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp]),
    'igr_att_softmax_bwd_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp,
                                               c_vp]),
    'igr_att_softmax_workspace_size': (c_i64, [_P(IgrCsr), c_i32]),
    'igr_att_softmax_ws_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp, c_i64,
                                              c_vp]),
    'igr_att_softmax_bwd_ws_f32': (ctypes.c_int, [_P(IgrCsr), c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp,
                                                  c_vp, c_i64, c_vp]),
    'igr_edge_dropout_f32': (ctypes.c_int, [c_i64, c_vp, c_vp, c_f32, c_vp, c_vp]),
    'igr_feat_values_f32': (ctypes.c_int, [c_i64, c_vp, c_vp, c_f32, c_vp, c_vp]),
    'igr_gather_rows_f32': (ctypes.c_int, [c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    'igr_scatter_add_rows_f32': (ctypes.c_int, [c_i64, c_i32, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp]),
    'igr_bpr_fwd_bwd_f32': (ctypes.c_int, [c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp,
                                           c_vp, c_vp, c_f32, c_f32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                                           c_vp]),
    'igr_bpr_workspace_floats': (c_i64, [c_i64, c_i32]),
    'igr_gemm_workspace_size': (c_i64, [c_i64, c_i64, c_i64]),
    'igr_gemm_f32': (ctypes.c_int, [c_i64, c_i64, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_vp, c_vp,
                                    c_i64, c_vp, c_i64, c_vp]),
    'igr_bpr_sample': (ctypes.c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, ctypes.c_uint64, ctypes.c_uint64,
                                      c_vp, c_i32, c_vp, c_vp, c_vp, c_vp]),
    'igr_adam_f32': (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_double, ctypes.c_double, c_i64, c_vp, c_vp]),
    'igr_adam_multi_f32': (ctypes.c_int, [c_i32, c_vp, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_double, c_vp, c_vp]),
    'igr_counter_add': (ctypes.c_int, [c_vp, c_i64, c_vp]),
    'igr_spmv_f32': (ctypes.c_int, [_P(IgrCsr), c_vp, c_vp, c_vp, c_vp]),
    'igr_layer_tail_f32': (ctypes.c_int, [c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, ctypes.c_float, ctypes.c_float,
                                          c_vp, c_vp, c_i64, c_vp, c_vp]),
    'igr_layer_tail_bwd_f32': (ctypes.c_int, [c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, ctypes.c_float,
                                              ctypes.c_float, c_vp, c_vp]),
    'igr_linear_wgrad_workspace_size': (c_i64, [c_i64, c_i32, c_i32]),
    'igr_linear_wgrad_f32': (ctypes.c_int, [c_i64, c_i32, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64,
                                            c_vp]),
    'igr_means_f32': (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    'igr_loss_combine_f32': (ctypes.c_int, [c_vp, c_vp, c_vp, c_f32, c_f32, c_f32, c_vp, c_vp, c_vp]),
}

_lib = None


class IgrError(RuntimeError):
    pass


def lib():
    """Load libigr.so once; raise if it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise IgrError(f'igr HIP library not found at {LIB_PATH}; build it with '
                           f'`python __graft_entry__.py` or inductive-recommendation_amd/build.py')
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc, what=''):
    if rc != 0:
        msg = lib().igr_last_error().decode(errors='replace')
        raise IgrError(f'{what or "igr"} failed (code {rc}): {msg}')


def call(name, *args):
    check(getattr(lib(), name)(*args), name)
