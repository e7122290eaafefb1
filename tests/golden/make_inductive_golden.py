"""Generate tests/golden/inductive.npz and inductive_ref_ckpt.pth by RUNNING the reference
through its inductive scenario: a model built on a dataset, saved, then moved to the same
dataset after new users and new items arrived.

The reference has no script for it, only the API (model.py:4208-4220 IGCN.save / load with
`generate_feat(..., is_updating=True)`, trainer.py:212-253 `inductive_eval`); the steps a
caller makes with that API are, on the reference's own objects:

    model = IGCN(cfg on the OLD dataset);  train;  model.save(path)
    model.config['dataset'] = full;  model.n_users, model.n_items = full.n_users, full.n_items
    model.norm_adj = model.generate_graph(full)
    model.load(path)            # embedding + maps + alpha, feature graph over the FULL dataset
    trainer = BasicTrainer(cfg on full, model);  trainer.inductive_eval(old.n_users, old.n_items)

The checkpoint is the file IGCN.save of the reference wrote (a dict of tensors, a float and two
dicts keyed by numpy int64 scalars); tests read it with igr.model.load_checkpoint (torch.load,
weights_only).  Same stubs for dgl / info_nce / torchmetrics as make_golden.py.

Run:  python tests/golden/make_inductive_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G  # noqa: E402  (installs the stubs, imports the reference)

ref_model, ref_trainer = G.ref_model, G.ref_trainer

N_OLD_USERS, N_OLD_ITEMS = 300, 200
N_USERS, N_ITEMS = 360, 250
N_EDGES, SEED = 4200, 21
D, L = 64, 2
TOPKS = [1, 5, 10, 20]


def main():
    torch.set_num_threads(4)
    edges = G.make_edges('uniform', N_USERS, N_ITEMS, N_EDGES, SEED)
    old_edges = edges[(edges[:, 0] < N_OLD_USERS) & (edges[:, 1] < N_OLD_ITEMS)]
    full = G.ToyDataset(N_USERS, N_ITEMS, edges, name='ind_full')
    old = G.ToyDataset(N_OLD_USERS, N_OLD_ITEMS, old_edges, name='ind_old')
    fx = {'n_users': np.int64(N_USERS), 'n_items': np.int64(N_ITEMS),
          'n_old_users': np.int64(N_OLD_USERS), 'n_old_items': np.int64(N_OLD_ITEMS),
          'train_array': edges.astype(np.int64), 'old_train_array': old_edges.astype(np.int64),
          'topks': np.array(TOPKS, np.int64)}
    for split in ['val', 'test']:
        data = getattr(full, split + '_data')
        fx[f'{split}_ptr'] = np.cumsum([0] + [len(x) for x in data]).astype(np.int64)
        fx[f'{split}_items'] = np.array(sum(data, []), dtype=np.int64)

    torch.manual_seed(900)
    m = ref_model.IGCN(G.model_cfg('IGCN', old, D, L))
    with torch.no_grad():
        m.w.mul_(1. + 0.1 * torch.randn(D, generator=torch.Generator().manual_seed(3)))  # w as after some training
    for _ in range(5):
        m.feat_mat_anneal()
    m.eval()
    with torch.no_grad():
        fx['old_rep'] = m.get_rep().numpy().copy()
    ckpt = os.path.join(HERE, 'inductive_ref_ckpt.pth')
    m.save(ckpt)
    fx['alpha'] = np.float64(m.alpha)
    fx['emb'] = m.embedding.weight.detach().numpy().copy()
    fx['w'] = m.w.detach().numpy().copy()

    # the dataset grows; the model follows it through the reference's own methods
    m.config['dataset'] = full
    m.n_users, m.n_items = full.n_users, full.n_items
    m.norm_adj = m.generate_graph(full)
    # the reference calls torch.load(path) as torch < 2.6 did; today's default (weights_only) reads
    # the file it has just written once the numpy-scalar names of the map keys are allowed
    import numpy.dtypes
    from numpy._core.multiarray import scalar
    with torch.serialization.safe_globals([scalar, np.dtype, numpy.dtypes.Int64DType]):
        m.load(ckpt)
    fi, fv = G.sp_np(m.feat_mat)
    fx['feat_idx'], fx['feat_val'] = fi, fv
    fx['feat_shape'] = np.array(m.feat_mat.shape, np.int64)
    fx['row_sum'] = m.row_sum.numpy().copy()
    ni_, nv_ = G.sp_np(m.norm_adj)
    fx['norm_idx'], fx['norm_val'] = ni_, nv_
    m.eval()
    with torch.no_grad():
        fx['rep'] = m.get_rep().numpy().copy()
        users = torch.arange(N_OLD_USERS - 8, N_OLD_USERS + 8)
        fx['predict_users'] = users.numpy()
        fx['predict_scores'] = m.predict(users).numpy().copy()

    tr = ref_trainer.BasicTrainer({'name': 'BasicTrainer', 'dataset': full, 'model': m, 'topks': TOPKS,
                                   'device': 'cpu', 'n_epochs': 0, 'test_batch_size': 64})
    seen = []
    plain_eval = tr.eval

    def recording_eval(*a, **kw):
        out = plain_eval(*a, **kw)
        seen.append(out[1])
        return out

    tr.eval = recording_eval
    tr.inductive_eval(N_OLD_USERS, N_OLD_ITEMS)
    assert len(seen) == 6
    for s, met in enumerate(seen):
        for mk in ['Precision', 'Recall', 'NDCG']:
            fx[f'slice{s}_{mk}'] = np.array([met[mk][k] for k in TOPKS], np.float64)
    path = os.path.join(HERE, 'inductive.npz')
    np.savez_compressed(path, **fx)
    print('wrote', path, os.path.getsize(path), 'and', ckpt, os.path.getsize(ckpt))
    for s, met in enumerate(seen):
        print(s, 'Recall@20', met['Recall'][20])


if __name__ == '__main__':
    main()
