"""Pin the CPU oracle against fixtures produced by running the reference.

Integer / index / degree arrays must match bit-exactly; fp32 values within the
tolerance stated per test.  (CPU only.)
"""
import numpy as np
import pytest

from oracle import igr_oracle as O

# fp32 tolerance for restatements whose summation order differs from the reference run:
# |y - ref| <= RTOL*|ref| + ATOL_ROW*max|ref_row|
RTOL, ATOL_ROW = 1e-5, 1e-6


def close(y, ref, rtol=RTOL, atol_row=ATOL_ROW):
    y = np.asarray(y, np.float64)
    ref = np.asarray(ref, np.float64)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    rowmax = np.abs(ref).max(axis=-1, keepdims=True) if ref.ndim > 1 else np.abs(ref).max()
    err = np.abs(y - ref)
    bound = rtol * np.abs(ref) + atol_row * rowmax + 1e-30
    worst = float((err / bound).max()) if err.size else 0.0
    assert worst <= 1.0, f'max err/bound = {worst:.3g}, max abs err {err.max():.3g}'


def graphs(fx):
    nu, ni, ta = int(fx['n_users']), int(fx['n_items']), fx['train_array']
    return nu, ni, ta, O.norm_adj(nu, ni, ta), O.generate_feat(nu, ni, ta)


def test_adjacency_bit_exact(golden):
    nu, ni, ta, A, F = graphs(golden)
    raw = O.generate_daj_mat(nu, ni, ta)
    np.testing.assert_array_equal(raw.row_ptr, golden['adj_indptr'])
    np.testing.assert_array_equal(raw.col, golden['adj_indices'])
    np.testing.assert_array_equal(raw.val, golden['adj_data'])  # duplicates summed -> 2.0
    np.testing.assert_array_equal(A.degree, golden['degree'])
    np.testing.assert_array_equal(A.dinv, golden['dinv'])
    # coalesced COO of norm_adj == CSR order (utils.py:38)
    np.testing.assert_array_equal(A.rows(), golden['norm_idx'][0])
    np.testing.assert_array_equal(A.col, golden['norm_idx'][1])
    np.testing.assert_array_equal(A.val, golden['norm_val'])  # (dinv[r]*a)*dinv[c], same host numpy


def test_feat_mat(golden):
    nu, ni, ta, A, F = graphs(golden)
    np.testing.assert_array_equal(np.array([F.n_rows, F.n_cols]), golden['feat_shape'])
    np.testing.assert_array_equal(F.rows(), golden['feat_idx'][0])
    np.testing.assert_array_equal(F.col, golden['feat_idx'][1])
    np.testing.assert_array_equal(F.row_sum, golden['row_sum'])
    # torch.pow(x, -0.5) lowers to rsqrt in the reference; numpy pow may differ by 1 ulp
    for tag, alpha in [('a1', 1.0), ('a099sq', float(golden['feat_alpha_a099sq'])),
                       ('a0', float(golden['feat_alpha_a0']))]:
        np.testing.assert_allclose(O.feat_values(F, alpha), golden['feat_val_' + tag], rtol=2e-7, atol=0)


def test_lightgcn_rep(golden):
    nu, ni, ta, A, F = graphs(golden)
    for d, L in [(32, 1), (64, 2)]:
        k = f'lgcn_d{d}_L{L}'
        close(O.lightgcn_rep(A, golden[k + '_emb'], L), golden[k + '_rep'])


def test_igcn_rep_and_grad(golden):
    nu, ni, ta, A, F = graphs(golden)
    fv = golden['feat_val_a1']
    for d, L in [(64, 2), (32, 3)]:
        k = f'igcn_d{d}_L{L}'
        emb = golden[k + '_emb']
        close(O.igcn_rep(A, F, fv, emb, L), golden[k + '_rep'])
        close(O.igcn_grad(A, F, fv, L, golden[k + '_R']), golden[k + '_grad'])
        # train-mode dropout with the reference's own uniform draws (model.py:4016-4028)
        fv_tr = O.dropout_values(fv, golden[k + '_train_rand'], 0.3)
        close(O.igcn_rep(A, F, fv_tr, emb, L), golden[k + '_train_rep'])


def test_imf_rep(golden):
    nu, ni, ta, A, F = graphs(golden)
    close(O.igcn_rep(A, F, golden['feat_val_a1'], golden['imf_emb'], 0), golden['imf_rep'])


def test_attigcn_forward(golden):
    nu, ni, ta, A, F = graphs(golden)
    g = golden
    x0, w = O.att_x0(F, g['att_feat_val'], g['att_emb'], g['att_wq'], g['att_bq'], g['att_wk'], g['att_bk'])
    close(w, g['att_alpha'], rtol=2e-5, atol_row=1e-6)
    close(x0, g['att_x0'], rtol=2e-5, atol_row=2e-6)


def test_bpr_terms(golden):
    nu, ni, ta, A, F = graphs(golden)
    k = 'igcn_d64_L2'
    rep = O.igcn_rep(A, F, golden['feat_val_a1'], golden[k + '_emb'], 2)
    w = np.ones(64, np.float32)
    l2, bpr, aux = O.bpr_terms(rep, golden[k + '_emb'], w, nu, nu, golden[k + '_bpr_users'],
                               golden[k + '_bpr_pos'], golden[k + '_bpr_neg'])
    close(l2, golden[k + '_bpr_l2'], rtol=1e-5)
    np.testing.assert_allclose(bpr, golden[k + '_bpr_loss'], rtol=1e-5)
    np.testing.assert_allclose(aux, golden[k + '_aux_loss'], rtol=1e-5)


def test_calculate_metrics(golden):
    topks = golden['eval_topks'].tolist()
    ptr, items = golden['test_ptr'], golden['test_items']
    test_data = [items[ptr[u]:ptr[u + 1]].tolist() for u in range(len(ptr) - 1)]
    res = O.calculate_metrics(test_data, golden['cm_rec_items'], topks)
    for mk in ['Precision', 'Recall', 'NDCG']:
        np.testing.assert_allclose([res[mk][k] for k in topks], golden['cm_' + mk], rtol=1e-6)


@pytest.mark.parametrize('split', ['val', 'test'])
def test_eval_metrics(golden, split):
    nu, ni, ta, A, F = graphs(golden)
    topks = golden['eval_topks'].tolist()
    rep = O.igcn_rep(A, F, golden['feat_val_a1'], golden['eval_emb'], 2)
    train_data = [[] for _ in range(nu)]
    for u, i in ta:
        train_data[u].append(int(i))
    ptr, items = golden[split + '_ptr'], golden[split + '_items']
    data = [items[ptr[u]:ptr[u + 1]].tolist() for u in range(nu)]
    if split == 'test':
        vptr, vit = golden['val_ptr'], golden['val_items']
        excl = [train_data[u] + vit[vptr[u]:vptr[u + 1]].tolist() for u in range(nu)]
    else:
        excl = train_data
    if max(len(set(e)) for e in excl) > ni - max(topks):
        pytest.skip('top-k reaches -inf ties; their order is torch.topk-internal')
    res = O.eval_metrics(rep, nu, excl, data, split, topks)
    for mk in ['Precision', 'Recall', 'NDCG']:
        np.testing.assert_allclose([res[mk][k] for k in topks], golden[f'eval_{split}_{mk}'], rtol=1e-6)
