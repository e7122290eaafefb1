"""Host-side logic of the model/trainer surface (CPU only)."""
import os

import numpy as np
import pytest

from igr import config as C
from igr import dataset as D
from igr import model as M
from igr import ops
from igr import trainer as T
from oracle import igr_oracle as O


def test_vectorised_calculate_metrics_matches_reference_fixture(golden):
    topks = golden['eval_topks'].tolist()
    ptr, items = golden['test_ptr'], golden['test_items']
    test_data = [items[ptr[u]:ptr[u + 1]].tolist() for u in range(len(ptr) - 1)]
    res = T.calculate_metrics(test_data, golden['cm_rec_items'], topks)
    for mk in ['Precision', 'Recall', 'NDCG']:
        np.testing.assert_allclose([res[mk][k] for k in topks], golden['cm_' + mk], rtol=1e-6)
    # the tensor form eval() uses on the device (here on CPU tensors): prefix sums, float64 averages
    import torch
    rec = golden['cm_rec_items']
    n_items = int(golden['n_items'])
    keys, lens = T.eval_keys(test_data, rec.shape[0], n_items)
    res = T.calculate_metrics_device(torch.from_numpy(keys), torch.from_numpy(lens), torch.from_numpy(rec), topks, n_items)
    for mk in ['Precision', 'Recall', 'NDCG']:
        np.testing.assert_allclose([res[mk][k] for k in topks], golden['cm_' + mk], rtol=1e-6)


def test_bpr_batch_sampler_semantics():
    rng = np.random.default_rng(0)
    pairs = np.stack([rng.integers(0, 50, 600), rng.integers(0, 40, 600)], 1)
    pairs = pairs[pairs[:, 0] % 7 != 3]  # some users without items

    class DS:
        n_users, n_items, train_pairs = 50, 40, pairs

        def __len__(self):
            return len(pairs)
    s = D.BPRBatchSampler(DS(), 128, seed=1)
    keys = set(map(tuple, pairs.tolist()))
    n = 0
    for u, p, q in s:
        n += len(u)
        assert all((a, b) in keys for a, b in zip(u, p))
        assert not any((a, b) in keys for a, b in zip(u, q))
        assert np.all(u % 7 != 3)
    assert n == len(pairs) and len(s) == (len(pairs) + 127) // 128


def test_reference_getitem_sampler():
    ds = D.BasicDataset({'name': 'x'})
    ds.n_users, ds.n_items = 3, 5
    ds.train_data = [[0, 1], [], [4]]
    for _ in range(50):
        u, p, n = ds[0][0]
        assert p in ds.train_data[u] and n not in ds.train_data[u]


def test_processed_dataset_roundtrip(tmp_path):
    ds = D.BasicDataset({'name': 'x'})
    ds.train_data = [[0, 2], [1], [3, 4, 0]]
    ds.val_data = [[1], [], [2]]
    ds.test_data = [[3], [0], []]
    ds.output_dataset(str(tmp_path))
    p = D.ProcessedDataset({'name': 'ProcessedDataset', 'path': str(tmp_path), 'device': 'cpu'})
    assert (p.n_users, p.n_items) == (3, 5)
    assert p.train_array == [[0, 0], [0, 2], [1, 1], [2, 3], [2, 4], [2, 0]]
    assert p.val_data == ds.val_data and p.test_data == ds.test_data


def test_config_tables_match_the_reference_row_by_row():
    """Every on-path row of the reference's five tables (config.py:1-527), at its index,
    with its hyper-parameters (tests/golden/make_config_golden.py dumped them); the other
    rows are None."""
    import json
    with open(os.path.join(os.path.dirname(__file__), 'golden', 'config_rows.json')) as f:
        ref = json.load(f)
    assert sorted(ref) == ['get_alibaba_config', 'get_amazon_config', 'get_gowalla_config', 'get_ml_config',
                           'get_yelp_config']
    for fn, want in ref.items():
        rows = getattr(C, fn)('DEVICE')
        assert len(rows) == want['n_rows']
        for k, row in enumerate(rows):
            if str(k) in want['rows']:
                assert [dict(x) for x in row] == want['rows'][str(k)], (fn, k)
            else:
                assert row is None, (fn, k)
    names = [m['name'] for _, m, _ in C.on_path(C.get_ml_config('cuda'))]
    assert names == ['LightGCN', 'IGCN', 'NGCF', 'IMF', 'IMCGAE']


def test_models_need_the_hip_device(golden):
    class DS:
        n_users, n_items = int(golden['n_users']), int(golden['n_items'])
        train_pairs = golden['train_array']
    with pytest.raises(ops.IgrError, match='no CPU fallback'):
        M.IGCN({'name': 'IGCN', 'embedding_size': 16, 'n_layers': 1, 'device': 'cpu', 'dropout': 0.3,
                'feature_ratio': 1., 'dataset': DS()})


def test_synthetic_pairs_reproducible():
    a = D.synthetic_pairs(1000, 100, 5000, seed=3)
    b = D.synthetic_pairs(1000, 100, 5000, seed=3)
    np.testing.assert_array_equal(a, b)
    assert a[:, 0].max() < 1000 and a[:, 1].max() < 100
    z = D.synthetic_pairs(1000, 100, 20000, seed=1, item_dist='zipf')
    c = np.bincount(z[:, 1], minlength=100)
    assert c[0] > 5 * c[50]


def test_rank_nodes_degree(golden):
    class DS:
        n_users, n_items = int(golden['n_users']), int(golden['n_items'])
        train_pairs = golden['train_array']
    ru, ri = M.graph_rank_nodes(DS(), 'degree')
    A = O.generate_daj_mat(DS.n_users, DS.n_items, DS.train_pairs)
    deg = O.row_sums(A)
    assert np.all(np.diff(deg[ru]) <= 0) and np.all(np.diff(deg[DS.n_users + ri]) <= 0)


def test_ngcf_graph_host_values_bit_exact(golden):
    """NGCF.generate_graph (model.py:4009-4014): adj + I, l1 row-normalised."""
    class DS:
        n_users, n_items = int(golden['n_users']), int(golden['n_items'])
        train_pairs = golden['train_array']
    m = M.NGCF({'name': 'NGCF', 'embedding_size': 8, 'layer_sizes': [8], 'device': 'cpu', 'dropout': 0.1,
                'dataset': DS()})
    h = m.norm_adj.host()
    np.testing.assert_array_equal(np.repeat(np.arange(m.norm_adj.n_rows), np.diff(h['row_ptr'])),
                                  golden['ngcf_norm_idx'][0])
    np.testing.assert_array_equal(h['col_idx'], golden['ngcf_norm_idx'][1])
    np.testing.assert_array_equal(m.norm_vals.numpy(), golden['ngcf_norm_val'])


@pytest.mark.parametrize('tag,min_inter', [('k5', 5), ('k10', 10)])
def test_gowalla_ingestion_matches_reference(tmp_path, tag, min_inter):
    """dataset.py:66-114 run by the reference on the same synthetic check-in file."""
    import os
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    import ml_like
    ml_like.write_checkins(os.path.join(tmp_path, 'Gowalla_totalCheckins.txt'))
    ref = np.load(os.path.join(GOLDEN, 'ingest_gowalla.npz'))
    ds = D.GowallaDataset({'name': 'GowallaDataset', 'path': str(tmp_path), 'device': 'cpu', 'min_inter': min_inter,
                           'split_ratio': [0.8, 0.1, 0.1]})
    assert [ds.n_users, ds.n_items] == ref[f'{tag}_n'].tolist()
    for split in ['train', 'val', 'test']:
        data = getattr(ds, split + '_data')
        np.testing.assert_array_equal(np.cumsum([0] + [len(x) for x in data]), ref[f'{tag}_{split}_ptr'])
        np.testing.assert_array_equal(np.array(sum(data, []), np.int64), ref[f'{tag}_{split}_items'])
    # round trip through the ProcessedDataset files the reference consumes
    ds.output_dataset(str(tmp_path / 'proc'))
    p = D.ProcessedDataset({'name': 'ProcessedDataset', 'path': str(tmp_path / 'proc'), 'device': 'cpu'})
    assert p.train_data == ds.train_data and p.n_users == ds.n_users


@pytest.mark.parametrize('tag,cls,fname,writer', [
    ('amazon', 'AmazonDataset', 'ratings_Books.csv', 'write_amazon_ratings'),
    ('yelp', 'YelpDataset', 'yelp_academic_dataset_review.json', 'write_yelp_reviews')])
@pytest.mark.parametrize('min_inter', [5, 10])
def test_amazon_yelp_ingestion_matches_reference(tmp_path, tag, cls, fname, writer, min_inter):
    """dataset.py:192-255 (string ids, rating > 3 filter, then dataset.py:66-114)
    run by the reference on the same synthetic files (tests/golden/make_ingest_golden.py)."""
    import os
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    import ml_like
    getattr(ml_like, writer)(os.path.join(tmp_path, fname))
    ref = np.load(os.path.join(GOLDEN, f'ingest_{tag}.npz'))
    ds = D.get_dataset({'name': cls, 'path': str(tmp_path), 'device': 'cpu', 'min_inter': min_inter,
                        'split_ratio': [0.8, 0.1, 0.1]})
    k = f'k{min_inter}'
    assert [ds.n_users, ds.n_items] == ref[f'{k}_n'].tolist()
    for split in ['train', 'val', 'test']:
        data = getattr(ds, split + '_data')
        np.testing.assert_array_equal(np.cumsum([0] + [len(x) for x in data]), ref[f'{k}_{split}_ptr'])
        np.testing.assert_array_equal(np.array(sum(data, []), np.int64), ref[f'{k}_{split}_items'])


def test_movielens_formats(tmp_path):
    rows = [(1, 10, 5, 100), (1, 20, 3, 50), (2, 10, 4, 70), (2, 30, 1, 10), (1, 30, 4, 20)] * 1
    with open(tmp_path / 'u.data', 'w') as f:
        for r in rows:
            f.write('\t'.join(map(str, r)) + '\n')
    ds = D.MovieLensDataset({'name': 'MovieLensDataset', 'path': str(tmp_path), 'min_inter': 1,
                             'split_ratio': [0.8, 0.1, 0.1]})
    assert (ds.n_users, ds.n_items) == (2, 3)
    # user 1: items by time: 30(20), 20(50), 10(100); n=3 -> train 2, test = whole list (quirk, n_test = 0)
    assert ds.train_data[0] == [2, 1] and ds.val_data[0] == [] and ds.test_data[0] == [2, 1, 0]
    os.makedirs(tmp_path / 'dat', exist_ok=True)
    with open(tmp_path / 'dat' / 'ratings.dat', 'w') as f:
        for r in rows:
            f.write('::'.join(map(str, r)) + '\n')
    d2 = D.MovieLensDataset({'name': 'MovieLensDataset', 'path': str(tmp_path / 'dat'), 'min_inter': 1,
                             'split_ratio': [0.8, 0.1, 0.1], 'min_rating': 4})
    assert d2.n_users == 2 and sum(len(x) for x in d2.train_data + d2.test_data) >= 3


def test_batch_edges_estimate_by_hand():
    """2 users, 3 items: u0-{i0,i1}, u1-{i1}; bipartite adjacency rows 0-1 users, 2-4 items.
    users: mean deg (2+1)/2; pos: u0 -> (deg i0 + deg i1)/2 = (1+2)/2, u1 -> deg i1 = 2
    => mean 1.75; neg: mean item deg (1+2+0)/3."""
    from igr import model as M
    row = np.array([0, 0, 1, 2, 3, 3])
    col = np.array([2, 3, 3, 0, 0, 1])
    rp = np.searchsorted(row, np.arange(6)).astype(np.int64)
    est = M.batch_edges_estimate(rp, col.astype(np.int32), 2, 10)
    assert est == pytest.approx(10 * (1.5 + 1.75 + 1.0))


def test_utils_graph_helpers_by_the_reference_names(golden):
    """utils.generate_daj_mat (utils.py:42-50) bit-exact; utils.get_sparse_tensor (33-39) of the
    matrix LightGCN.generate_graph forms (model.py:89-98) carries the reference's values in
    its coalesced order."""
    import scipy.sparse as sp
    from igr import utils

    class DS:
        n_users, n_items = int(golden['n_users']), int(golden['n_items'])
        train_array = golden['train_array'].tolist()
    adj = utils.generate_daj_mat(DS())
    assert adj.dtype == np.float32 and adj.shape == (DS.n_users + DS.n_items,) * 2
    np.testing.assert_array_equal(adj.indptr, golden['adj_indptr'])
    np.testing.assert_array_equal(adj.indices, golden['adj_indices'])
    np.testing.assert_array_equal(adj.data, golden['adj_data'])
    degree = np.array(np.sum(adj, axis=1)).squeeze()
    degree = np.maximum(1., degree)
    d = sp.diags(np.power(degree, -0.5), format='csr', dtype=np.float32)
    g = utils.get_sparse_tensor(d.dot(adj).dot(d), 'cpu')
    h = g.host()
    np.testing.assert_array_equal(np.repeat(np.arange(g.n_rows), np.diff(h['row_ptr'])), golden['norm_idx'][0])
    np.testing.assert_array_equal(h['col_idx'], golden['norm_idx'][1])
    np.testing.assert_array_equal(g.values.numpy(), golden['norm_val'])
    # a second set of values over the same graph is a view: one reverse graph, base untouched
    v2 = g.values * 2
    g2 = g.with_values(v2)
    assert g2.values is v2 and g.values is not v2 and g2.reverse() is g.reverse() and g2.csr is g.csr


def test_trainer_record_writes_every_metric_at_every_k():
    """BasicTrainer.record (trainer.py:49-56)."""
    import types
    seen = []
    writer = types.SimpleNamespace(add_scalar=lambda tag, v, step: seen.append((tag, v, step)))
    me = types.SimpleNamespace(topks=[1, 5], model=types.SimpleNamespace(name='IGCN'), name='IGCNTrainer', epoch=3)
    T.BasicTrainer.record(me, writer, 'validation', {'Recall': {1: .1, 5: .5}, 'NDCG': {1: .2, 5: .6}})
    assert seen == [('IGCN_IGCNTrainer/validation_Recall@1', .1, 3), ('IGCN_IGCNTrainer/validation_Recall@5', .5, 3),
                    ('IGCN_IGCNTrainer/validation_NDCG@1', .2, 3), ('IGCN_IGCNTrainer/validation_NDCG@5', .6, 3)]


def test_auxiliary_dataset_restricts_and_renumbers():
    """AuxiliaryDataset (dataset.py:258-273) against its definition, with maps that
    cover part of the users / items in shuffled order (feature_ratio < 1)."""
    rng = np.random.RandomState(4)
    nu, ni = 40, 30

    lists = [rng.permutation(ni)[:rng.randint(0, 9)].tolist() for _ in range(nu)]

    class DS:
        n_users, n_items, device = nu, ni, 'cpu'
        train_data = lists
        train_array = [[u, i] for u in range(nu) for i in lists[u]]

        def __len__(self):
            return len(self.train_array)
    user_map = {int(u): k for k, u in enumerate(rng.permutation(nu)[:25])}
    item_map = {int(i): k for k, i in enumerate(rng.permutation(ni)[:18])}
    aux = D.AuxiliaryDataset(DS(), user_map, item_map)
    want = [[] for _ in range(len(user_map))]
    for o_user in range(nu):
        if o_user in user_map:
            want[user_map[o_user]] += [item_map[i] for i in DS.train_data[o_user] if i in item_map]
    assert (aux.n_users, aux.n_items, len(aux)) == (25, 18, len(DS.train_array))
    assert aux.train_data == want
    assert sorted(aux.train_pairs.tolist()) == sorted([u, i] for u in range(25) for i in want[u])
    ident = D.AuxiliaryDataset(DS(), {u: u for u in range(nu)}, {i: i for i in range(ni)})
    assert ident.train_data == DS.train_data
    empty = D.AuxiliaryDataset(DS(), {}, {})
    assert (empty.n_users, empty.n_items, empty.train_data, len(empty.train_pairs)) == (0, 0, [], 0)


def test_utils_keeps_the_names_reference_code_imports():
    """utils.py:280-305: AverageMeter and Unbuffered are imported by name by code written
    against the reference."""
    import io
    from igr.utils import AverageMeter, Unbuffered
    m = AverageMeter()
    m.update(2.0, 3)
    m.update(4.0, 1)
    assert m.sum == 10.0 and m.count == 4 and m.avg == 2.5
    buf = io.StringIO()
    flushed = []
    buf.flush = lambda: flushed.append(len(buf.getvalue()))
    w = Unbuffered(buf)
    w.write('ab')
    w.writelines(['c', 'd'])
    assert buf.getvalue() == 'abcd' and flushed == [2, 4] and w.closed is False
