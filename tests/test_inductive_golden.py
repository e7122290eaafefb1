"""The inductive scenario, CPU side: a model built on a dataset, saved by the reference
(IGCN.save, model.py:4208-4211), then moved to the dataset after new users and items
arrived (IGCN.load -> generate_feat(is_updating=True), model.py:4213-4220) and scored over
the six slices of BasicTrainer.inductive_eval (trainer.py:212-253).  The fixture and the
checkpoint come from running the reference (tests/golden/make_inductive_golden.py).
Pins the oracle's restatement and the checkpoint reader.  (CPU only.)
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import igr_oracle as O
from test_oracle_golden import close

CKPT = os.path.join(GOLDEN, 'inductive_ref_ckpt.pth')


@pytest.fixture(scope='module')
def fx():
    with np.load(os.path.join(GOLDEN, 'inductive.npz')) as z:
        return {k: z[k] for k in z.files}


def lists(fx, split):
    ptr, items = fx[split + '_ptr'], fx[split + '_items']
    return [items[ptr[u]:ptr[u + 1]].tolist() for u in range(int(fx['n_users']))]


def test_reference_checkpoint_reads_with_the_restricted_loader(fx):
    from igr.model import load_checkpoint
    p = load_checkpoint(CKPT, 'cpu')
    assert sorted(p) == ['alpha', 'item_map', 'sate_dict', 'user_map']
    assert sorted(p['sate_dict']) == ['embedding.weight', 'w']
    np.testing.assert_array_equal(p['sate_dict']['embedding.weight'].numpy(), fx['emb'])
    np.testing.assert_array_equal(p['sate_dict']['w'].numpy(), fx['w'])
    assert float(p['alpha']) == float(fx['alpha'])
    nu0, ni0 = int(fx['n_old_users']), int(fx['n_old_items'])
    assert {int(k): int(v) for k, v in p['user_map'].items()} == {u: u for u in range(nu0)}
    assert {int(k): int(v) for k, v in p['item_map'].items()} == {i: i for i in range(ni0)}


def test_checkpoint_loader_refuses_code(tmp_path):
    """Anything beyond tensors, numbers, dicts and numpy integer scalars is refused, not run."""
    import pickle

    import torch
    from igr.model import load_checkpoint

    class Payload:
        def __reduce__(self):
            return (os.getcwd, ())

    path = tmp_path / 'bad.pth'
    torch.save({'sate_dict': {}, 'user_map': Payload()}, path)
    with pytest.raises(pickle.UnpicklingError):
        load_checkpoint(str(path), 'cpu')


def test_oracle_moves_the_feature_graph_to_the_grown_dataset(fx):
    nu, ni = int(fx['n_users']), int(fx['n_items'])
    nu0, ni0 = int(fx['n_old_users']), int(fx['n_old_items'])
    umap, imap = {u: u for u in range(nu0)}, {i: i for i in range(ni0)}
    F = O.generate_feat(nu, ni, fx['train_array'], umap, imap)
    np.testing.assert_array_equal(np.array([F.n_rows, F.n_cols]), fx['feat_shape'])
    assert F.n_cols == nu0 + ni0 + 2  # the table of the old dataset: no row for a new user or item
    np.testing.assert_array_equal(F.rows(), fx['feat_idx'][0])
    np.testing.assert_array_equal(F.col, fx['feat_idx'][1])
    np.testing.assert_array_equal(F.row_sum, fx['row_sum'])
    fv = O.feat_values(F, float(fx['alpha']))
    np.testing.assert_allclose(fv, fx['feat_val'], rtol=2e-7, atol=0)
    A = O.norm_adj(nu, ni, fx['train_array'])
    np.testing.assert_array_equal(A.val, fx['norm_val'])
    rep = O.igcn_rep(A, F, fx['feat_val'], fx['emb'], 2)
    close(rep, fx['rep'])
    # on the old dataset the same maps are the identity: generate_feat without them
    F0 = O.generate_feat(nu0, ni0, fx['old_train_array'])
    F1 = O.generate_feat(nu0, ni0, fx['old_train_array'], umap, imap)
    np.testing.assert_array_equal(F0.col, F1.col)
    np.testing.assert_array_equal(F0.row_ptr, F1.row_ptr)
    A0 = O.norm_adj(nu0, ni0, fx['old_train_array'])
    close(O.igcn_rep(A0, F0, O.feat_values(F0, float(fx['alpha'])), fx['emb'], 2), fx['old_rep'])


def test_oracle_inductive_eval_slices(fx):
    nu, ni = int(fx['n_users']), int(fx['n_items'])
    topks = fx['topks'].tolist()
    train = [[] for _ in range(nu)]
    for u, i in fx['train_array']:
        train[u].append(int(i))
    val, test = lists(fx, 'val'), lists(fx, 'test')
    excl = [a + b for a, b in zip(train, val)]
    res = O.inductive_eval(fx['rep'].copy(), nu, ni, excl, test, int(fx['n_old_users']), int(fx['n_old_items']), topks)
    for s, name in enumerate(O.INDUCTIVE_SLICES):
        for mk in ['Precision', 'Recall', 'NDCG']:
            np.testing.assert_allclose([res[name][mk][k] for k in topks], fx[f'slice{s}_{mk}'], rtol=1e-6,
                                       err_msg=f'{name} {mk}')


def test_oracle_imcgae_rep():
    """IMCGAE.get_rep (model.py:4313-4339) restated in the oracle against the reference run
    (tests/golden/make_imcgae_golden.py), eval mode and train mode - the train-mode masks are
    the draws F.dropout makes from the CPU generator at the fixture's seed."""
    import torch
    import torch.nn.functional as F
    with np.load(os.path.join(GOLDEN, 'imcgae.npz')) as z:
        g = {k: z[k] for k in z.files}
    L, p = int(g['n_layers']), float(g['dropout'])
    for cname in ['uni', 'pow']:
        with np.load(os.path.join(GOLDEN, cname + '.npz')) as z:
            nu, ni, ta = int(z['n_users']), int(z['n_items']), z['train_array']
        A = O.norm_adj(nu, ni, ta)
        close(O.imcgae_rep(A, g[cname + '_emb'], nu, ni, L), g[cname + '_rep'])
        torch.manual_seed(int(g['train_seed']))
        masks = [F.dropout(torch.ones(nu + ni), p=p - 0.1 * i, training=True).numpy() for i in range(L)]
        close(O.imcgae_rep(A, g[cname + '_emb'], nu, ni, L, masks), g[cname + '_train_rep'])
