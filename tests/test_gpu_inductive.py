"""The inductive scenario on the GPU: igr.model.IGCN reads a checkpoint the REFERENCE wrote
on the old dataset, follows the dataset to its grown form with the reference's own call
sequence (config['dataset'], n_users / n_items, generate_graph, load -> generate_feat with
is_updating=True; model.py:4208-4220) and reports BasicTrainer.inductive_eval's six slices
(trainer.py:212-253).  Expected values: the reference run of
tests/golden/make_inductive_golden.py.  Tolerances as in test_gpu_models."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from igr import model as M
from igr import trainer as T
from test_gpu_kernels import close

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda')
CKPT = os.path.join(GOLDEN, 'inductive_ref_ckpt.pth')
SLICES = ['All users and all items', 'Old users and all items', 'New users and all items',
          'All users and old items', 'All users and new items', 'Old users and old items']


@pytest.fixture(scope='module')
def fx():
    with np.load(os.path.join(GOLDEN, 'inductive.npz')) as z:
        return {k: z[k] for k in z.files}


class DS:
    def __init__(self, name, n_users, n_items, pairs, val=None, test=None):
        self.name, self.n_users, self.n_items = name, n_users, n_items
        self.train_pairs = pairs
        self.train_array = pairs.tolist()
        self.train_data = [[] for _ in range(n_users)]
        for u, i in pairs:
            self.train_data[u].append(int(i))
        self.val_data = val if val is not None else [[] for _ in range(n_users)]
        self.test_data = test if test is not None else [[] for _ in range(n_users)]

    def __len__(self):
        return len(self.train_array)


def datasets(fx):
    nu, ni = int(fx['n_users']), int(fx['n_items'])
    split = lambda s: [fx[s + '_items'][fx[s + '_ptr'][u]:fx[s + '_ptr'][u + 1]].tolist() for u in range(nu)]  # noqa: E731
    old = DS('ind_old', int(fx['n_old_users']), int(fx['n_old_items']), fx['old_train_array'])
    full = DS('ind_full', nu, ni, fx['train_array'], split('val'), split('test'))
    return old, full


def moved_model(fx):
    old, full = datasets(fx)
    torch.manual_seed(1)
    m = M.IGCN({'name': 'IGCN', 'embedding_size': 64, 'n_layers': 2, 'device': DEV, 'dropout': 0.3,
                'feature_ratio': 1., 'dataset': old})
    m.load(CKPT)  # the file IGCN.save of the reference wrote
    m.eval()
    with torch.no_grad():
        old_rep = m.get_rep().cpu().numpy()
    # the dataset grows; the call sequence a user of the reference writes
    m.config['dataset'] = full
    m.n_users, m.n_items = full.n_users, full.n_items
    m.norm_adj = m.generate_graph(full)
    m.load(CKPT)
    return m, full, old_rep


def test_reference_checkpoint_then_grown_dataset(fx):
    m, full, old_rep = moved_model(fx)
    assert m.alpha == float(fx['alpha'])
    np.testing.assert_array_equal(m.embedding.weight.detach().cpu().numpy(), fx['emb'])
    np.testing.assert_array_equal(m.w.detach().cpu().numpy(), fx['w'])
    close(old_rep, fx['old_rep'])
    F = m.feat_mat
    h = F.host()
    assert [F.n_rows, F.n_cols] == fx['feat_shape'].tolist()
    np.testing.assert_array_equal(np.repeat(np.arange(F.n_rows), np.diff(h['row_ptr'])), fx['feat_idx'][0])
    np.testing.assert_array_equal(h['col_idx'], fx['feat_idx'][1])
    np.testing.assert_array_equal(m.row_sum.cpu().numpy(), fx['row_sum'])
    np.testing.assert_allclose(m.feat_vals.cpu().numpy(), fx['feat_val'], rtol=2e-7, atol=0)
    np.testing.assert_array_equal(m.norm_vals.cpu().numpy(), fx['norm_val'])
    m.eval()
    with torch.no_grad():
        rep = m.get_rep()
        close(rep.cpu().numpy(), fx['rep'])
        users = torch.from_numpy(fx['predict_users']).to(DEV)
        close(m.predict(users).cpu().numpy(), fx['predict_scores'], rtol=2e-5, atol_row=2e-6)


def test_inductive_eval_slices_match_reference(fx, capsys):
    m, full, _ = moved_model(fx)
    topks = fx['topks'].tolist()
    tr = T.BasicTrainer({'name': 'BasicTrainer', 'dataset': full, 'model': m, 'topks': topks, 'device': DEV,
                         'n_epochs': 0, 'test_batch_size': 64})
    before = [list(x) for x in full.test_data]
    res = tr.inductive_eval(int(fx['n_old_users']), int(fx['n_old_items']))
    assert full.test_data == before  # left as found
    assert list(res) == SLICES
    lines = capsys.readouterr().out.strip().splitlines()
    assert [ln.split(' result. ')[0] for ln in lines] == SLICES
    for s, name in enumerate(SLICES):
        for mk in ['Precision', 'Recall', 'NDCG']:
            np.testing.assert_allclose([res[name][mk][k] for k in topks], fx[f'slice{s}_{mk}'], rtol=1e-6,
                                       err_msg=f'{name} {mk}')


def test_eval_sees_edited_lists_outside_train(fx):
    """Outside train() nothing is cached: editing dataset.test_data in place (as the
    reference's inductive_eval does, trainer.py:219-220) changes the next eval."""
    m, full, _ = moved_model(fx)
    topks = fx['topks'].tolist()
    tr = T.BasicTrainer({'name': 'BasicTrainer', 'dataset': full, 'model': m, 'topks': topks, 'device': DEV,
                         'n_epochs': 0, 'test_batch_size': 64})
    _, met_all, prot = tr.eval('test')
    assert prot == []
    for u in range(int(fx['n_old_users']), full.n_users):
        full.test_data[u] = []
    _, met_old, _ = tr.eval('test')
    np.testing.assert_allclose([met_all['Recall'][k] for k in topks], fx['slice0_Recall'], rtol=1e-6)
    np.testing.assert_allclose([met_old['Recall'][k] for k in topks], fx['slice1_Recall'], rtol=1e-6)
