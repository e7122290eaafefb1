"""Golden fixtures at the size of BASELINE's configurations, by RUNNING the reference.

    att_ml1m      the reference's AttIGCN (model.py:4223-4287, dead text evaluated as in
                  make_golden.py) on the MovieLens-1M shape: 6,040 x 3,706, ~800 K train
                  interactions, d = 64, 2 layers, 4 heads
    igcn_gowalla  the reference's IGCN (model.py:4107-4220) on the Gowalla shape:
                  29,858 x 40,981, ~1.04 M train interactions, d = 128, 3 layers

The interaction data comes from tests/golden/ml_like.py and the parameters from
numpy RandomState streams (`scale_params`), so the tests rebuild the identical
inputs and the fixtures hold only OUTPUTS: full-tensor float64 column sums and the
values at a fixed sample of rows / edges (a few hundred KB per configuration).

Run (build container only; the GPU box never sees /root/reference):
    python tests/golden/make_scale_golden.py [att_ml1m] [igcn_gowalla]
"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ml_like  # noqa: E402
from ml_like import scale_cotangent as P_R, scale_params, scale_samples  # noqa: E402

import make_golden as MG  # noqa: E402  (installs the dgl / info_nce / torchmetrics stand-ins, imports the reference)


class DS:
    def __init__(self, name, n_users, n_items, train):
        self.name, self.n_users, self.n_items, self.device = name, n_users, n_items, 'cpu'
        self.train_data = train
        self.train_array = [[u, i] for u in range(n_users) for i in train[u]]

    def __len__(self):
        return len(self.train_array)


def summarize(fx, key, t, rows):
    """Column sums (float64), the sum of |x|, and the sampled rows of a [n, d] tensor."""
    a = t.detach().numpy()
    fx[key + '_colsum'] = a.astype(np.float64).sum(0)
    fx[key + '_abssum'] = np.float64(np.abs(a.astype(np.float64)).sum())
    fx[key + '_rows'] = a[rows].copy()


def att_ml1m():
    shape = 'ml1m'
    nu, ni, _, d, L, _ = ml_like.SHAPES[shape]
    train, _, _ = ml_like.splits_for(shape)
    ds = DS(shape, nu, ni, train)
    AttIGCN = MG.load_attigcn()
    t0 = time.time()
    m = AttIGCN(MG.model_cfg('AttIGCN', ds, d, L))
    P = scale_params('att_ml1m', m.embedding.weight.shape[0], d, heads=4)
    with torch.no_grad():
        m.embedding.weight.copy_(torch.from_numpy(P['emb']))
        m.weight_q.weight.copy_(torch.from_numpy(P['wq']))
        m.weight_q.bias.copy_(torch.from_numpy(P['bq']))
        m.weight_k.weight.copy_(torch.from_numpy(P['wk']))
        m.weight_k.bias.copy_(torch.from_numpy(P['bk']))
    nnz = m.feat_mat._nnz()
    S = scale_samples('att_ml1m', nu + ni, nnz)
    fx = {'n_train': np.int64(len(ds)), 'nnz_feat': np.int64(nnz)}
    m.eval()
    alpha = m.inductive_rep_layer(m.feat_mat, return_alpha=True)
    fx['alpha_sum'] = np.float64(alpha.detach().double().sum())
    fx['alpha_edges'] = alpha.detach().numpy()[S['edges']].copy()
    x0 = m.inductive_rep_layer(m.feat_mat)
    summarize(fx, 'x0', x0, S['rows'])
    rep = m.get_rep()
    summarize(fx, 'rep', rep, S['rows'])
    R = torch.from_numpy(P_R(rep.shape))
    (rep * R).sum().backward()
    summarize(fx, 'grad_emb', m.embedding.weight.grad, S['feat_rows'])
    fx['grad_wq'] = m.weight_q.weight.grad.numpy().copy()
    fx['grad_wk'] = m.weight_k.weight.grad.numpy().copy()
    fx['grad_bq'] = m.weight_q.bias.grad.numpy().copy()
    # train mode: dropout removes edges before the softmax (model.py:4016-4028), draws from the CPU generator
    m.train()
    torch.manual_seed(33)
    with torch.no_grad():
        summarize(fx, 'train_rep', m.get_rep(), S['rows'])
    np.savez_compressed(os.path.join(HERE, 'scale_att_ml1m.npz'), **fx)
    print(f'att_ml1m: nnz_feat {nnz}, {time.time() - t0:.0f}s, '
          f'{os.path.getsize(os.path.join(HERE, "scale_att_ml1m.npz"))} bytes', flush=True)


def igcn_gowalla():
    shape = 'gowalla'
    nu, ni, _, d, L, _ = ml_like.SHAPES[shape]
    train, _, _ = ml_like.splits_for(shape)
    ds = DS(shape, nu, ni, train)
    t0 = time.time()
    m = MG.ref_model.IGCN(MG.model_cfg('IGCN', ds, d, L))
    P = scale_params('igcn_gowalla', m.embedding.weight.shape[0], d)
    with torch.no_grad():
        m.embedding.weight.copy_(torch.from_numpy(P['emb']))
    S = scale_samples('igcn_gowalla', nu + ni, m.feat_mat._nnz(), m.norm_adj._nnz())
    fx = {'n_train': np.int64(len(ds)), 'nnz_feat': np.int64(m.feat_mat._nnz()),
          'nnz_adj': np.int64(m.norm_adj._nnz())}
    fx['norm_val_sum'] = np.float64(m.norm_adj.values().double().sum())
    fx['norm_val_edges'] = m.norm_adj.values().numpy()[S['adj_edges']].copy()
    m.eval()
    rep = m.get_rep()
    summarize(fx, 'rep', rep, S['rows'])
    (rep * torch.from_numpy(P_R(rep.shape))).sum().backward()
    summarize(fx, 'grad_emb', m.embedding.weight.grad, S['feat_rows'])
    m.train()
    torch.manual_seed(31)
    with torch.no_grad():
        summarize(fx, 'train_rep', m.get_rep(), S['rows'])
    np.savez_compressed(os.path.join(HERE, 'scale_igcn_gowalla.npz'), **fx)
    print(f'igcn_gowalla: nnz_adj {int(fx["nnz_adj"])}, {time.time() - t0:.0f}s, '
          f'{os.path.getsize(os.path.join(HERE, "scale_igcn_gowalla.npz"))} bytes', flush=True)


if __name__ == '__main__':
    torch.set_num_threads(4)
    for name in (sys.argv[1:] or ['att_ml1m', 'igcn_gowalla']):
        {'att_ml1m': att_ml1m, 'igcn_gowalla': igcn_gowalla}[name]()
