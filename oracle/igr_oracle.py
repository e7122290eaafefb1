"""igr_oracle - CPU restatement of the reference hot path (numpy + oracle.c).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker.  The product package
(inductive-recommendation_amd/igr) never imports this module.

Pinned against tests/golden/*.npz, which tests/golden/make_golden.py produced
by running the reference code itself (see tests/test_oracle_golden.py).
Every function cites the reference file:line it restates
(/root/reference/<file>:<line>).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, 'build', 'liboracle.so')
_lib = None

_i64p = np.ctypeslib.ndpointer(np.int64, flags='C_CONTIGUOUS')
_f32p = np.ctypeslib.ndpointer(np.float32, flags='C_CONTIGUOUS')
_f64p = np.ctypeslib.ndpointer(np.float64, flags='C_CONTIGUOUS')


class _Nullable:
    """ctypes argtype accepting None or a contiguous numpy array of one dtype."""

    def __init__(self, dtype):
        self.dtype = dtype

    def from_param(self, obj):
        if obj is None:
            return None
        assert obj.dtype == self.dtype and obj.flags['C_CONTIGUOUS'], (obj.dtype, self.dtype)
        return obj.ctypes.data_as(ctypes.c_void_p)


def build():
    subprocess.check_call(['make', '-s', '-C', _HERE, 'build/liboracle.so'])


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH) or \
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, 'oracle.c')):
        build()
    L = ctypes.CDLL(_LIB_PATH)
    i64, i32 = ctypes.c_int64, ctypes.c_int
    L.orc_coo_to_csr.restype = i64
    L.orc_coo_to_csr.argtypes = [i64, i64, i64, _i64p, _i64p, _Nullable(np.float32), i32,
                                 _i64p, _i64p, _f32p, _Nullable(np.int64)]
    L.orc_spmm_sum_f32.restype = None
    L.orc_spmm_sum_f32.argtypes = [i64, i64, _i64p, _i64p, _Nullable(np.float32), _Nullable(np.int64),
                                   _f32p, i64, _f32p, i64, i32]
    L.orc_spmm_sum_f64.restype = None
    L.orc_spmm_sum_f64.argtypes = [i64, i64, _i64p, _i64p, _Nullable(np.float32), _Nullable(np.int64),
                                   _f32p, i64, _f64p, i64]
    L.orc_sddmm_dot_f32.restype = None
    L.orc_sddmm_dot_f32.argtypes = [i64, i64, i64, _i64p, _i64p, _Nullable(np.int64), _f32p, _f32p, _f32p]
    L.orc_segment_reduce_f32.restype = None
    L.orc_segment_reduce_f32.argtypes = [i64, i64, _i64p, _Nullable(np.int64), _f32p, i32, _f32p]
    L.orc_att_softmax_f32.restype = None
    L.orc_att_softmax_f32.argtypes = [i64, i64, _i64p, _Nullable(np.int64), _f32p, ctypes.c_float, _f32p]
    _lib = L
    return L


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


# --------------------------------------------------------------------------- graph construction

class CSR:
    def __init__(self, n_rows, n_cols, row_ptr, col, val, eid=None):
        self.n_rows, self.n_cols = int(n_rows), int(n_cols)
        self.row_ptr, self.col, self.val, self.eid = row_ptr, col, val, eid

    @property
    def nnz(self):
        return int(self.row_ptr[-1])

    def rows(self):
        return np.repeat(np.arange(self.n_rows, dtype=np.int64), np.diff(self.row_ptr))

    def transpose(self):
        """Reverse graph used by the gspmm backward: (col, row) CSR, eid -> CSR position of self."""
        t = coo_to_csr(self.n_cols, self.n_rows, self.col, self.rows(), None, dedup=False)
        t.val = None if self.val is None else self.val[t.eid]
        return t


def coo_to_csr(n_rows, n_cols, row, col, val=None, dedup=True):
    """scipy coo_matrix(...).tocsr() + torch coalesce (utils.py:33-50) when dedup;
    a DGL multigraph in CSR order when not (model.py:4183)."""
    row, col = _c(row, np.int64), _c(col, np.int64)
    nnz = len(row)
    rp = np.zeros(n_rows + 1, np.int64)
    co = np.zeros(max(nnz, 1), np.int64)
    vo = np.zeros(max(nnz, 1), np.float32)
    eid = np.zeros(max(nnz, 1), np.int64)
    v = None if val is None else _c(val, np.float32)
    n = lib().orc_coo_to_csr(n_rows, n_cols, nnz, row, col, v, int(dedup), rp, co, vo, eid)
    return CSR(n_rows, n_cols, rp, co[:n].copy(), vo[:n].copy(), eid[:n].copy())


def row_sums(A):
    """np.sum(mat, axis=1) of an integer-valued float32 matrix (exact below 2**24)."""
    return np.bincount(A.rows(), weights=A.val, minlength=A.n_rows).astype(np.float32)


def generate_daj_mat(n_users, n_items, train_array):
    """utils.py:42-50: symmetric bipartite adjacency, duplicates summed."""
    ta = np.asarray(train_array, dtype=np.int64).reshape(-1, 2)
    u, i = ta[:, 0], ta[:, 1]
    row = np.concatenate([u, i + n_users])
    col = np.concatenate([i + n_users, u])
    n = n_users + n_items
    return coo_to_csr(n, n, row, col, None, dedup=True)


def norm_adj(n_users, n_items, train_array):
    """LightGCN.generate_graph (model.py:89-98): D^-1/2 A D^-1/2 in float32.
    degree = float32 row sum; dinv = np.power(max(1, deg), -0.5) (float32);
    value = (dinv[r] * a) * dinv[c] (sp.diags(.).dot(A).dot(diags))."""
    A = generate_daj_mat(n_users, n_items, train_array)
    deg = row_sums(A)
    dinv = np.power(np.maximum(np.float32(1.), deg), np.float32(-0.5)).astype(np.float32)
    r = A.rows()
    A.val = ((dinv[r] * A.val).astype(np.float32) * dinv[A.col]).astype(np.float32)
    A.degree, A.dinv = deg, dinv
    return A


def generate_feat(n_users, n_items, train_array, user_map=None, item_map=None):
    """IGCN.generate_feat (model.py:4139-4175).
    user u -> column U' + item_map[i] for each training item i in item_map; item i ->
    column user_map[u] for each training user u in user_map; every user -> column
    U' + I'; every item -> column U' + I' + 1 (U', I' = the sizes of the maps).
    Maps None: feature_ratio = 1 on this dataset (identity maps, 4147-4156); maps
    given: is_updating=True (4157-4159) - the maps of the dataset the model was
    built on, applied to a dataset that has grown since.  row_sum = row degree."""
    ta = np.asarray(train_array, dtype=np.int64).reshape(-1, 2)
    u, i = ta[:, 0], ta[:, 1]
    U, I = n_users, n_items
    umap = np.arange(U, dtype=np.int64) if user_map is None else np.full(U, -1, np.int64)
    imap = np.arange(I, dtype=np.int64) if item_map is None else np.full(I, -1, np.int64)
    for m, table in ((user_map, umap), (item_map, imap)):
        if m is not None:
            for k, v in m.items():
                table[int(k)] = int(v)
    Ud = U if user_map is None else len(user_map)
    Id = I if item_map is None else len(item_map)
    ki, ku = imap[i] >= 0, umap[u] >= 0
    row = np.concatenate([u[ki], U + i[ku], np.arange(U), U + np.arange(I)])
    col = np.concatenate([Ud + imap[i[ki]], umap[u[ku]], np.full(U, Ud + Id), np.full(I, Ud + Id + 1)])
    F = coo_to_csr(U + I, Ud + Id + 2, row, col, None, dedup=True)
    F.row_sum = row_sums(F)
    return F


def feat_values(F, alpha):
    """IGCN.update_feat_mat (model.py:4127-4130): row_sum[row] ** ((alpha-1)/2 - 0.5)."""
    e = (alpha - 1.) / 2. - 0.5
    return np.power(F.row_sum[F.rows()], np.float32(e)).astype(np.float32)


def dropout_values(val, rand, p):
    """NGCF.dropout_sp_mat (model.py:4016-4028) as a value mask over the fixed CSR:
    keep = floor((1 - p) + U[0,1)); kept values divided by (1 - p); dropped -> 0.
    Summing a 0.0 term is exact, so this equals removing the edge."""
    keep = np.floor(np.float32(1. - p) + rand.astype(np.float32)).astype(bool)
    return np.where(keep, (val / np.float32(1. - p)).astype(np.float32), np.float32(0.)).astype(np.float32)


# --------------------------------------------------------------------------- propagation

def spmm(A, x, val=None, n_threads=1):
    """gspmm(g, 'mul', 'sum', x, val) over CSR A (float accumulator, edge order)."""
    x = _c(x, np.float32)
    d = x.shape[1]
    out = np.zeros((A.n_rows, d), np.float32)
    v = A.val if val is None else _c(val, np.float32)
    lib().orc_spmm_sum_f32(A.n_rows, d, A.row_ptr, A.col, v, None, x, d, out, d, n_threads)
    return out


def spmm64(A, x, val=None):
    x = _c(x, np.float32)
    d = x.shape[1]
    out = np.zeros((A.n_rows, d), np.float64)
    v = A.val if val is None else _c(val, np.float32)
    lib().orc_spmm_sum_f64(A.n_rows, d, A.row_ptr, A.col, v, None, x, d, out, d)
    return out


def lightgcn_rep(A, emb, n_layers):
    """LightGCN.get_rep (model.py:100-110): mean of [E, AE, ..., A^L E]."""
    reps = [emb.astype(np.float32)]
    x = reps[0]
    for _ in range(n_layers):
        x = spmm(A, x)
        reps.append(x)
    return np.stack(reps).mean(0).astype(np.float32)


def imcgae_rep(A, emb, n_users, n_items, n_layers, masks=None):
    """IMCGAE.get_rep (model.py:4313-4339) as written there: rows [personal | general |
    identical] (3 d wide), each layer x <- A (mask_i * x), rep = x_0 + sum_i x_{i+1} / (i + 2).
    masks: per layer a node-dropout mask (F.dropout of ones) or None (eval mode)."""
    n = n_users + n_items
    ident, gen_u, gen_i = emb[n], emb[n + 1], emb[n + 2]
    x = np.concatenate([np.concatenate([emb[:n_users], np.tile(gen_u, (n_users, 1)), np.tile(ident, (n_users, 1))], 1),
                        np.concatenate([emb[n_users:n], np.tile(gen_i, (n_items, 1)), np.tile(ident, (n_items, 1))], 1)],
                       0).astype(np.float32)
    rep = x.copy()
    for i in range(n_layers):
        if masks is not None and masks[i] is not None:
            x = x * masks[i][:, None]
        x = spmm(A, x)
        rep = rep + x / np.float32(i + 2)
    return rep


def igcn_rep(A, F, fvals, emb, n_layers):
    """IGCN.get_rep (model.py:4188-4200) with inductive_rep_layer (4177-4186)."""
    x0 = spmm(F, emb, val=fvals)
    reps = [x0]
    x = x0
    for _ in range(n_layers):
        x = spmm(A, x)
        reps.append(x)
    return np.stack(reps).mean(0).astype(np.float32)


def igcn_grad(A, F, fvals, n_layers, g):
    """d/dEmb of sum(igcn_rep * G): gspmm backward = reverse-graph SpMM (model.py:106, 4196)."""
    L1 = n_layers + 1
    dx = (g / np.float32(L1)).astype(np.float32)
    for _ in range(n_layers):
        dx = (g / np.float32(L1) + spmm(A.transpose(), dx)).astype(np.float32)
    Ft = F.transpose()
    return spmm(Ft, dx, val=fvals[Ft.eid])


def sddmm_dot(A, q, k):
    """AttIGCN.masked_mm (model.py:4246-4255)."""
    n, h, d = q.shape
    out = np.zeros((A.nnz, h), np.float32)
    lib().orc_sddmm_dot_f32(A.n_rows, h, d, A.row_ptr, A.col, None, _c(q, np.float32), _c(k, np.float32), out)
    return out


def segment_reduce(A, x, reduce):
    """gspmm(g, 'copy_rhs', 'sum'|'max', None, x) (model.py:4270, 4273)."""
    x = _c(x, np.float32)
    h = 1 if x.ndim == 1 else x.shape[1]
    out = np.zeros((A.n_rows, h), np.float32)
    lib().orc_segment_reduce_f32(A.n_rows, h, A.row_ptr, None, x, 1 if reduce == 'max' else 0, out)
    return out


def att_softmax(A, alpha, d):
    """AttIGCN.inductive_rep_layer steps 4-7 (model.py:4270-4275)."""
    alpha = _c(alpha, np.float32)
    w = np.zeros(A.nnz, np.float32)
    lib().orc_att_softmax_f32(A.n_rows, alpha.shape[1], A.row_ptr, None, alpha, np.float32(np.sqrt(d)), w)
    return w


def linear(x, w, b):
    return (x.astype(np.float32) @ w.T.astype(np.float32) + b).astype(np.float32)


def att_x0(F, fvals, emb, wq, bq, wk, bk, n_heads=4):
    """AttIGCN.inductive_rep_layer (model.py:4257-4281), eval mode."""
    d = emb.shape[1]
    xk = linear(emb, wk, bk).reshape(-1, n_heads, d)
    xq = linear(spmm(F, emb, val=fvals), wq, bq).reshape(-1, n_heads, d)
    alpha = sddmm_dot(F, xq, xk)
    w = att_softmax(F, alpha, d)
    return spmm(F, emb, val=w), w


# --------------------------------------------------------------------------- training / eval terms

def softplus(x):
    x = x.astype(np.float64)
    return np.where(x > 20, x, np.log1p(np.exp(np.minimum(x, 20))))


def bpr_terms(rep, emb, w, n_users, n_feat_users, users, pos, neg):
    """NGCF.bpr_forward (model.py:4046-4052) + IGCNTrainer loss (trainer.py:535-551)."""
    ur, pr, nr = rep[users], rep[n_users + pos], rep[n_users + neg]
    l2 = (ur ** 2).sum(1) + (pr ** 2).sum(1) + (nr ** 2).sum(1)
    bpr = softplus((ur * nr).sum(1) - (ur * pr).sum(1)).mean()
    ue, pe, ne = emb[users], emb[n_feat_users + pos], emb[n_feat_users + neg]
    aux = softplus((ue * ne * w).sum(1) - (ue * pe * w).sum(1)).mean()
    return l2.astype(np.float32), np.float32(bpr), np.float32(aux)


def calculate_metrics(eval_data, rec_items, topks):
    """BasicTrainer.calculate_metrics (trainer.py:115-144)."""
    hit = np.zeros(rec_items.shape, np.float32)
    for u in range(rec_items.shape[0]):
        s = set(eval_data[u])
        for j in range(rec_items.shape[1]):
            if rec_items[u, j] in s:
                hit[u, j] = 1.
    n_eval = np.array([len(x) for x in eval_data], np.int32)
    res = {'Precision': {}, 'Recall': {}, 'NDCG': {}}
    for k in topks:
        hn = hit[:, :k].sum(1)
        with np.errstate(invalid='ignore', divide='ignore'):
            rec = hn / n_eval
        mh = np.minimum(n_eval, k)
        mhm = (np.arange(k)[None, :] < mh[:, None]).astype(np.float32)
        den = np.log2(np.arange(2, k + 2, dtype=np.float32))[None, :]
        dcg = (hit[:, :k] / den).sum(1)
        idcg = (mhm / den).sum(1)
        with np.errstate(invalid='ignore', divide='ignore'):
            ndcg = dcg / idcg
        m = mh > 0
        res['Precision'][k] = (hn / k)[m].mean()
        res['Recall'][k] = rec[m].mean()
        res['NDCG'][k] = ndcg[m].mean()
    return res


def eval_metrics(rep, n_users, train_data, eval_data, split, topks, banned_items=None):
    """BasicTrainer.eval (trainer.py:146-170) with LightGCN.predict (model.py:122-127):
    scores = rep[u] . rep[items]^T; train items (and val items for 'test') set to -inf
    except for split 'train'; banned items set to -inf for every user (166-167);
    top-max(topks); then calculate_metrics."""
    scores = rep[:n_users] @ rep[n_users:].T
    if split != 'train':
        for u in range(n_users):
            scores[u, train_data[u]] = -np.inf
    if banned_items is not None:
        scores[:, banned_items] = -np.inf
    kmax = max(topks)
    rec = np.argsort(-scores, axis=1, kind='stable')[:, :kmax]
    return calculate_metrics(eval_data, rec, topks)


INDUCTIVE_SLICES = ['All users and all items', 'Old users and all items', 'New users and all items',
                    'All users and old items', 'All users and new items', 'Old users and old items']


def inductive_eval(rep, n_users, n_items, exclude, test_data, n_old_users, n_old_items, topks):
    """BasicTrainer.inductive_eval (trainer.py:212-253): the 'test' metrics over six
    slices of the test lists, in the order of INDUCTIVE_SLICES.  `exclude` = train + val
    lists (what eval('test') masks)."""
    olds = [[i for i in x if i < n_old_items] for x in test_data]
    news = [[i for i in x if i >= n_old_items] for x in test_data]
    cut = lambda lists, keep: [x if keep(u) else [] for u, x in enumerate(lists)]  # noqa: E731
    ban_new, ban_old = np.arange(n_old_items, n_items), np.arange(n_old_items)
    cases = [(test_data, None),
             (cut(test_data, lambda u: u < n_old_users), None),
             (cut(test_data, lambda u: u >= n_old_users), None),
             (olds, ban_new), (news, ban_old),
             (cut(olds, lambda u: u < n_old_users), ban_new)]
    return {name: eval_metrics(rep, n_users, exclude, data, 'test', topks, banned)
            for name, (data, banned) in zip(INDUCTIVE_SLICES, cases)}
