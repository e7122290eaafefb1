"""Train the REFERENCE IGCN on MovieLens-shaped data and record its trajectory.

Runs /root/reference's IGCN model (model.py:4107-4220) and its
BasicTrainer.eval / calculate_metrics (trainer.py:115-210), with the per-batch
loss code of IGCNTrainer.train_one_epoch (trainer.py:535-556) applied to
fixed batches from tests/golden/ml_like.py instead of the DataLoader's random
worker sampling, so that igr can be driven with the identical batches,
identical CPU-generator dropout draws and identical initialisation.

DGL is absent; `dgl.ops.gspmm(g,'mul','sum')` is restated as
a CSR SpMM whose backward is the transposed SpMM (DGL's gspmm semantics; the
edge values never require grad on this path).  Writes
tests/golden/train_<shape>.npz (IGCN) and, with `lightgcn`, the reference
LightGCN under BPRTrainer's loss to tests/golden/train_lgcn_<shape>.npz.
Run: python tests/golden/make_train_golden.py [shape ...]
     python tests/golden/make_train_golden.py lightgcn [shape ...]
     python tests/golden/make_train_golden.py imf [shape ...]    (-> train_imf_<shape>.npz)
     python tests/golden/make_train_golden.py ngcf [shape ...]   (-> train_ngcf_<shape>.npz)
     python tests/golden/make_train_golden.py imcgae [shape ...] (-> train_imcgae_<shape>.npz)
"""
import os
import sys
import time
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ml_like  # noqa: E402

REF = '/root/reference'


class _CsrSpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A, At, x):
        ctx.At = At
        return torch.sparse.mm(A, x)

    @staticmethod
    def backward(ctx, dy):
        return None, None, torch.sparse.mm(ctx.At, dy)


def install_stubs():
    dgl = types.ModuleType('dgl')
    ops = types.ModuleType('dgl.ops')

    class _G:
        def __init__(self, edges, n):
            self.src, self.dst, self.n = edges[0], edges[1], n

    def graph(edges, num_nodes=None, device=None):
        return _G(edges, num_nodes)

    cache = {}

    def gspmm(g, op, reduce, lhs_data=None, rhs_data=None):
        # (column, row) come from a coalesced COO, so dst is sorted: CSR order already
        assert op == 'mul' and reduce == 'sum' and not rhs_data.requires_grad
        key = (g.dst.data_ptr(), g.src.data_ptr(), rhs_data.data_ptr(), rhs_data._version, g.n)
        if key not in cache:
            if len(cache) > 8:
                cache.clear()
            m = lhs_data.shape[0]
            crow = torch.zeros(g.n + 1, dtype=torch.int64)
            crow[1:] = torch.cumsum(torch.bincount(g.dst, minlength=g.n), 0)
            A = torch.sparse_csr_tensor(crow, g.src, rhs_data, (g.n, m))
            order = torch.argsort(g.src, stable=True)
            tcrow = torch.zeros(m + 1, dtype=torch.int64)
            tcrow[1:] = torch.cumsum(torch.bincount(g.src, minlength=m), 0)
            At = torch.sparse_csr_tensor(tcrow, g.dst[order], rhs_data[order], (m, g.n))
            cache[key] = (A, At, rhs_data)  # keep rhs alive so its data_ptr stays unique
        A, At, _ = cache[key]
        return _CsrSpMM.apply(A, At, lhs_data)

    dgl.graph, ops.gspmm, dgl.ops = graph, gspmm, ops
    sys.modules['dgl'], sys.modules['dgl.ops'] = dgl, ops
    inf = types.ModuleType('info_nce')
    inf.InfoNCE = object
    sys.modules['info_nce'] = inf
    tm, tmf = types.ModuleType('torchmetrics'), types.ModuleType('torchmetrics.functional')
    tmf.pairwise_cosine_similarity = None
    tm.functional = tmf
    sys.modules['torchmetrics'], sys.modules['torchmetrics.functional'] = tm, tmf


class DS:
    def __init__(self, name, n_users, n_items, train, val, test):
        self.name, self.n_users, self.n_items, self.device = name, n_users, n_items, 'cpu'
        self.train_data, self.val_data, self.test_data = train, val, test
        self.train_array = [[u, i] for u in range(n_users) for i in train[u]]

    def __len__(self):
        return len(self.train_array)


def run(shape, imf=False):
    """imf: the reference's IMF (model.py:4290-4297; config row 6: the inductive layer alone,
    dropout 0.1, l2_reg 1e-5, aux_reg 0.1) under the same IGCNTrainer loop, six epochs,
    to train_imf_<shape>.npz."""
    install_stubs()
    sys.path.insert(0, REF)
    import model as ref_model
    import trainer as ref_trainer
    nu, ni, mean_deg, d, L, epochs = ml_like.SHAPES[shape]
    if imf:
        L, epochs = 0, 6
    train, val, test = ml_like.splits_for(shape)
    ds = DS(shape, nu, ni, train, val, test)
    bs = 2048
    spe = ml_like.steps_per_epoch(train, bs)
    main_b = ml_like.batches_for(shape, train, ni, bs, spe * epochs, seed=1)
    aux_b = ml_like.batches_for(shape, train, ni, bs, spe * epochs, seed=2)  # feature_ratio = 1: aux maps are identity
    torch.manual_seed(7)
    cfg = {'name': 'IMF' if imf else 'IGCN', 'embedding_size': d, 'n_layers': L, 'device': 'cpu',
           'dropout': 0.1 if imf else 0.3, 'feature_ratio': 1., 'dataset': ds}
    m = (ref_model.IMF if imf else ref_model.IGCN)(cfg)
    init_sum = float(m.embedding.weight.detach().double().sum())
    init_abs = float(m.embedding.weight.detach().double().abs().sum())
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    topks = [20]
    tr = ref_trainer.BasicTrainer({'name': 'BasicTrainer', 'dataset': ds, 'model': m, 'topks': [1, 5, 10, 15, 20],
                                   'device': 'cpu', 'n_epochs': 0, 'test_batch_size': 512})
    l2_reg, aux_reg = (1.e-5, 0.1) if imf else (0., 0.01)
    losses, val_rec, val_ndcg, test_rec = [], [], [], []
    step_loss = []
    t0 = time.time()
    for ep in range(epochs):
        m.train()
        tot = 0.
        for s in range(spe):
            u, p, n = (torch.from_numpy(a) for a in main_b[ep * spe + s])
            # trainer.py:536-556
            users_r, pos_items_r, neg_items_r, l2_norm_sq = m.bpr_forward(u, p, n)
            pos_scores = torch.sum(users_r * pos_items_r, dim=1)
            neg_scores = torch.sum(users_r * neg_items_r, dim=1)
            bpr_loss = F.softplus(neg_scores - pos_scores).mean()
            au, ap, an = (torch.from_numpy(a) for a in aux_b[ep * spe + s])
            users_r = m.embedding(au)
            pos_items_r = m.embedding(ap + len(m.user_map))
            neg_items_r = m.embedding(an + len(m.user_map))
            pos_scores = torch.sum(users_r * pos_items_r * m.w[None, :], dim=1)
            neg_scores = torch.sum(users_r * neg_items_r * m.w[None, :], dim=1)
            aux_loss = F.softplus(neg_scores - pos_scores).mean()
            reg_loss = l2_reg * l2_norm_sq.mean() + aux_reg * aux_loss
            loss = bpr_loss + reg_loss
            opt.zero_grad()
            loss.backward()
            opt.step()
            tot += loss.item()
            if ep == 0 and s < 20:
                step_loss.append(loss.item())
        m.feat_mat_anneal()
        losses.append(tot / spe)
        _, met, _ = tr.eval('val')
        val_rec.append(met['Recall'][20])
        val_ndcg.append(met['NDCG'][20])
        _, met, _ = tr.eval('test')
        test_rec.append(met['Recall'][20])
        print(f'{shape} epoch {ep}: loss {losses[-1]:.5f} val R@20 {val_rec[-1]:.4f} '
              f'test R@20 {test_rec[-1]:.4f} ({time.time() - t0:.0f}s)', flush=True)
    np.savez_compressed(os.path.join(HERE, f'train_imf_{shape}.npz' if imf else f'train_{shape}.npz'),
                        losses=np.array(losses), val_recall20=np.array(val_rec),
                        val_ndcg20=np.array(val_ndcg), test_recall20=np.array(test_rec),
                        first_step_losses=np.array(step_loss), init_sum=init_sum, init_abs=init_abs,
                        seed=7, epochs=epochs, d=d, n_layers=L, alpha_final=m.alpha)


def run_lightgcn(shape, l2_reg=1e-4):
    """The reference LightGCN (model.py:79-127) under BPRTrainer's loss
    (trainer.py:412-429) on the same fixed batches; no dropout on this path."""
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import model as ref_model
    import trainer as ref_trainer
    nu, ni, mean_deg, d, L, epochs = ml_like.SHAPES[shape]
    train, val, test = ml_like.splits_for(shape)
    ds = DS(shape, nu, ni, train, val, test)
    bs = 2048
    spe = ml_like.steps_per_epoch(train, bs)
    main_b = ml_like.batches_for(shape, train, ni, bs, spe * epochs, seed=1)
    torch.manual_seed(11)
    m = ref_model.LightGCN({'name': 'LightGCN', 'embedding_size': d, 'n_layers': L, 'device': 'cpu',
                            'dataset': ds})
    init_sum = float(m.embedding.weight.detach().double().sum())
    init_abs = float(m.embedding.weight.detach().double().abs().sum())
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    tr = ref_trainer.BasicTrainer({'name': 'BasicTrainer', 'dataset': ds, 'model': m, 'topks': [1, 5, 10, 15, 20],
                                   'device': 'cpu', 'n_epochs': 0, 'test_batch_size': 512})
    losses, val_rec, test_rec, step_loss = [], [], [], []
    t0 = time.time()
    for ep in range(epochs):
        m.train()
        tot = 0.
        for s in range(spe):
            u, p, n = (torch.from_numpy(a) for a in main_b[ep * spe + s])
            users_r, pos_items_r, neg_items_r, l2_norm_sq = m.bpr_forward(u, p, n)
            pos_scores = torch.sum(users_r * pos_items_r, dim=1)
            neg_scores = torch.sum(users_r * neg_items_r, dim=1)
            loss = F.softplus(neg_scores - pos_scores).mean() + l2_reg * l2_norm_sq.mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
            tot += loss.item()
            if ep == 0 and s < 20:
                step_loss.append(loss.item())
        losses.append(tot / spe)
        _, met, _ = tr.eval('val')
        val_rec.append(met['Recall'][20])
        _, met, _ = tr.eval('test')
        test_rec.append(met['Recall'][20])
        print(f'lgcn {shape} epoch {ep}: loss {losses[-1]:.5f} val R@20 {val_rec[-1]:.4f} '
              f'test R@20 {test_rec[-1]:.4f} ({time.time() - t0:.0f}s)', flush=True)
    np.savez_compressed(os.path.join(HERE, f'train_lgcn_{shape}.npz'), losses=np.array(losses),
                        val_recall20=np.array(val_rec), test_recall20=np.array(test_rec),
                        first_step_losses=np.array(step_loss), init_sum=init_sum, init_abs=init_abs, seed=11,
                        epochs=epochs, d=d, n_layers=L, l2_reg=l2_reg)


def run_ngcf(shape, l2_reg=1e-3, epochs=6):
    """The reference NGCF (model.py:3986-4055, config row 4: layer_sizes [d, d, d], l2_reg 1e-3)
    under BPRTrainer's loss (trainer.py:412-429) on the same fixed batches, dropout 0 (the
    edge mask and F.dropout are then the identity, so no random draw separates the runs)."""
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import model as ref_model
    import trainer as ref_trainer
    nu, ni, mean_deg, d, L, _ = ml_like.SHAPES[shape]
    train, val, test = ml_like.splits_for(shape)
    ds = DS(shape, nu, ni, train, val, test)
    bs = 2048
    spe = ml_like.steps_per_epoch(train, bs)
    main_b = ml_like.batches_for(shape, train, ni, bs, spe * epochs, seed=1)
    torch.manual_seed(13)
    m = ref_model.NGCF({'name': 'NGCF', 'embedding_size': d, 'layer_sizes': [d, d, d], 'device': 'cpu',
                        'dropout': 0., 'dataset': ds})
    init = {k: (float(v.detach().double().sum()), float(v.detach().double().abs().sum()))
            for k, v in m.named_parameters()}
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    tr = ref_trainer.BasicTrainer({'name': 'BasicTrainer', 'dataset': ds, 'model': m, 'topks': [1, 5, 10, 15, 20],
                                   'device': 'cpu', 'n_epochs': 0, 'test_batch_size': 512})
    losses, val_rec, test_rec, step_loss = [], [], [], []
    t0 = time.time()
    for ep in range(epochs):
        m.train()
        tot = 0.
        for s in range(spe):
            u, p, n = (torch.from_numpy(a) for a in main_b[ep * spe + s])
            users_r, pos_items_r, neg_items_r, l2_norm_sq = m.bpr_forward(u, p, n)
            pos_scores = torch.sum(users_r * pos_items_r, dim=1)
            neg_scores = torch.sum(users_r * neg_items_r, dim=1)
            loss = F.softplus(neg_scores - pos_scores).mean() + l2_reg * l2_norm_sq.mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
            tot += loss.item()
            if ep == 0 and s < 20:
                step_loss.append(loss.item())
        losses.append(tot / spe)
        _, met, _ = tr.eval('val')
        val_rec.append(met['Recall'][20])
        _, met, _ = tr.eval('test')
        test_rec.append(met['Recall'][20])
        print(f'ngcf {shape} epoch {ep}: loss {losses[-1]:.5f} val R@20 {val_rec[-1]:.4f} '
              f'test R@20 {test_rec[-1]:.4f} ({time.time() - t0:.0f}s)', flush=True)
    names = sorted(init)
    np.savez_compressed(os.path.join(HERE, f'train_ngcf_{shape}.npz'), losses=np.array(losses),
                        val_recall20=np.array(val_rec), test_recall20=np.array(test_rec),
                        first_step_losses=np.array(step_loss), param_names=np.array(names),
                        init_sum=np.array([init[k][0] for k in names]), init_abs=np.array([init[k][1] for k in names]),
                        seed=13, epochs=epochs, d=d, l2_reg=l2_reg)


def run_imcgae(shape, epochs=6):
    """The reference IMCGAE (model.py:4300-4345, config row 7: 3 layers, dropout 0.3, l2_reg 0)
    under BPRTrainer's loss on the same fixed batches; its node-dropout masks are the CPU
    generator's draws (three F.dropout calls per step), which igr replays with
    dropout_rng = 'cpu'."""
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import model as ref_model
    import trainer as ref_trainer
    nu, ni, mean_deg, d, _, _ = ml_like.SHAPES[shape]
    train, val, test = ml_like.splits_for(shape)
    ds = DS(shape, nu, ni, train, val, test)
    bs = 2048
    spe = ml_like.steps_per_epoch(train, bs)
    main_b = ml_like.batches_for(shape, train, ni, bs, spe * epochs, seed=1)
    torch.manual_seed(17)
    m = ref_model.IMCGAE({'name': 'IMCGAE', 'embedding_size': d, 'n_layers': 3, 'device': 'cpu', 'dropout': 0.3,
                          'dataset': ds})
    e = m.embedding.weight.detach().double()
    init_sum, init_abs = float(e.sum()), float(e.abs().sum())
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    tr = ref_trainer.BasicTrainer({'name': 'BasicTrainer', 'dataset': ds, 'model': m, 'topks': [1, 5, 10, 15, 20],
                                   'device': 'cpu', 'n_epochs': 0, 'test_batch_size': 512})
    losses, val_rec, test_rec, step_loss = [], [], [], []
    t0 = time.time()
    for ep in range(epochs):
        m.train()
        tot = 0.
        for s in range(spe):
            u, p, n = (torch.from_numpy(a) for a in main_b[ep * spe + s])
            users_r, pos_items_r, neg_items_r, l2_norm_sq = m.bpr_forward(u, p, n)
            loss = F.softplus(torch.sum(users_r * neg_items_r, dim=1) - torch.sum(users_r * pos_items_r, dim=1)).mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
            tot += loss.item()
            if ep == 0 and s < 20:
                step_loss.append(loss.item())
        losses.append(tot / spe)
        _, met, _ = tr.eval('val')
        val_rec.append(met['Recall'][20])
        _, met, _ = tr.eval('test')
        test_rec.append(met['Recall'][20])
        print(f'imcgae {shape} epoch {ep}: loss {losses[-1]:.5f} val R@20 {val_rec[-1]:.4f} '
              f'test R@20 {test_rec[-1]:.4f} ({time.time() - t0:.0f}s)', flush=True)
    np.savez_compressed(os.path.join(HERE, f'train_imcgae_{shape}.npz'), losses=np.array(losses),
                        val_recall20=np.array(val_rec), test_recall20=np.array(test_rec),
                        first_step_losses=np.array(step_loss), init_sum=init_sum, init_abs=init_abs, seed=17,
                        epochs=epochs, d=d, n_layers=3, dropout=0.3)


if __name__ == '__main__':
    args = sys.argv[1:]
    if args and args[0] == 'lightgcn':
        for sh in (args[1:] or ['ml100k']):
            run_lightgcn(sh)
    elif args and args[0] == 'imf':
        for sh in (args[1:] or ['ml100k']):
            run(sh, imf=True)
    elif args and args[0] == 'ngcf':
        for sh in (args[1:] or ['ml100k']):
            run_ngcf(sh)
    elif args and args[0] == 'imcgae':
        for sh in (args[1:] or ['ml100k']):
            run_imcgae(sh)
    else:
        for sh in (args or list(ml_like.SHAPES)):
            run(sh)
