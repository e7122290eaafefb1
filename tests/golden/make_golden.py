"""Generate the golden fixtures under tests/golden/ by RUNNING the reference.

This script is the only place that touches /root/reference.  It runs in the
build container (never on the GPU box, never from pytest) and writes small
.npz fixtures that the tests read.

How the reference is run
------------------------
`/root/reference/{utils,dataset,model,trainer}.py` are imported as-is.  Three
third-party modules they import at top level are absent from the image and
are registered in `sys.modules` before the import:

* `dgl` (DGL >= 0.8, README.md:8, no pinned version).  Only `dgl.graph` and
  `dgl.ops.gspmm` are reached on the hot path.  `gspmm` is restated from DGL's
  published semantics: out[dst] = reduce_{e: src->dst} lhs[src] (op) rhs[e];
  zero-in-degree rows give 0 for both sum and max.  The 'mul'/'sum' form is
  the `index_add_` restatement the survey verified; 'copy_rhs'/'max' uses
  `scatter_reduce(amax, include_self=False)` on a zero tensor.
* `info_nce`, `torchmetrics.functional` - only used by out-of-scope SGL/DOSE.

Consequence: every fixture pins the reference's own graph construction
(utils.generate_daj_mat, LightGCN.generate_graph, IGCN.generate_feat,
update_feat_mat, dropout_sp_mat), its layer composition (padding, slicing,
stack/mean), BPR gathers and the metric code (trainer.calculate_metrics,
BasicTrainer.eval).  The SpMM arithmetic itself is DGL's and is pinned by the
restated semantics above plus a float64 scipy cross-check.

AttIGCN (model.py:4223-4287) is dead code inside a string literal; this
script evaluates that class text against the imported `model` module
namespace so its forward can be pinned too.

Run:  python tests/golden/make_golden.py
"""
import ast
import json
import os
import sys
import types

import numpy as np
import torch

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


def install_stubs():
    dgl = types.ModuleType('dgl')
    ops = types.ModuleType('dgl.ops')

    class _G:
        def __init__(self, edges, num_nodes):
            self.src, self.dst = edges
            self.n = num_nodes

    def graph(edges, num_nodes=None, device=None):
        return _G(edges, num_nodes)

    def gspmm(g, op, reduce, lhs_data=None, rhs_data=None):
        if op == 'mul' and reduce == 'sum':
            r = rhs_data if rhs_data.dim() == lhs_data.dim() else rhs_data[:, None]
            out = torch.zeros(g.n, lhs_data.shape[1], dtype=lhs_data.dtype)
            return out.index_add(0, g.dst, lhs_data[g.src] * r)
        if op == 'copy_rhs':
            shape = (g.n,) + tuple(rhs_data.shape[1:])
            out = torch.zeros(shape, dtype=rhs_data.dtype)
            idx = g.dst.view(-1, *([1] * (rhs_data.dim() - 1))).expand_as(rhs_data)
            if reduce == 'sum':
                return out.scatter_add(0, idx, rhs_data)
            if reduce == 'max':
                return out.scatter_reduce(0, idx, rhs_data, reduce='amax', include_self=False)
        raise NotImplementedError((op, reduce))

    dgl.graph = graph
    ops.gspmm = gspmm
    dgl.ops = ops
    sys.modules['dgl'] = dgl
    sys.modules['dgl.ops'] = ops
    inf = types.ModuleType('info_nce')
    inf.InfoNCE = object
    sys.modules['info_nce'] = inf
    tm = types.ModuleType('torchmetrics')
    tmf = types.ModuleType('torchmetrics.functional')
    tmf.pairwise_cosine_similarity = None
    tm.functional = tmf
    sys.modules['torchmetrics'] = tm
    sys.modules['torchmetrics.functional'] = tmf


install_stubs()
sys.path.insert(0, REF)
import model as ref_model  # noqa: E402
import trainer as ref_trainer  # noqa: E402
import utils as ref_utils  # noqa: E402


def load_attigcn():
    """Evaluate the AttIGCN class text (model.py:4223-4287) in model's namespace."""
    src = open(os.path.join(REF, 'model.py')).read()
    tree = ast.parse(src)
    for node in tree.body:
        if isinstance(node, ast.Expr) and isinstance(node.value, ast.Constant) \
                and isinstance(node.value.value, str) and 'class AttIGCN' in node.value.value:
            ns = vars(ref_model)
            exec(compile(node.value.value, 'model.py:AttIGCN', 'exec'), ns)
            return ns['AttIGCN']
    raise RuntimeError('AttIGCN text not found')


class ToyDataset:
    """Stands in for ProcessedDataset: the attributes the models/trainers read."""

    def __init__(self, n_users, n_items, train_array, name='toy'):
        self.name = name
        self.n_users = n_users
        self.n_items = n_items
        self.device = 'cpu'
        self.train_array = [list(map(int, p)) for p in train_array]
        self.train_data = [[] for _ in range(n_users)]
        for u, i in self.train_array:
            self.train_data[u].append(i)
        rng = np.random.RandomState(n_users + n_items)
        self.val_data = [sorted(set(rng.randint(0, n_items, size=rng.randint(0, 4)).tolist()))
                         for _ in range(n_users)]
        self.test_data = [sorted(set(rng.randint(0, n_items, size=rng.randint(0, 5)).tolist()))
                          for _ in range(n_users)]


def make_edges(kind, n_users, n_items, n_edges, seed):
    rng = np.random.RandomState(seed)
    if kind == 'uniform':
        u = rng.randint(0, n_users, size=n_edges)
        i = rng.randint(0, n_items, size=n_edges)
    elif kind == 'powerlaw':
        u = rng.randint(0, n_users, size=n_edges)
        w = 1.0 / np.arange(1, n_items + 1) ** 1.1
        i = rng.choice(n_items, size=n_edges, p=w / w.sum())
    else:
        raise ValueError(kind)
    return np.stack([u, i], axis=1)


def toy_edges():
    # 7 users x 5 items; user 6 and item 4 isolated; (0,1) duplicated.
    return np.array([[0, 0], [0, 1], [0, 1], [1, 1], [1, 2], [2, 0], [2, 3], [3, 3],
                     [4, 0], [4, 1], [4, 2], [4, 3], [5, 2]], dtype=np.int64)


CASES = {
    # name: (n_users, n_items, edges-spec)
    'toy': (7, 5, None),
    'uni': (300, 200, ('uniform', 3000, 11)),
    'pow': (500, 400, ('powerlaw', 8000, 12)),
}


def model_cfg(name, ds, d, L, **kw):
    cfg = {'name': name, 'embedding_size': d, 'n_layers': L, 'device': 'cpu',
           'dropout': 0.3, 'feature_ratio': 1., 'dataset': ds}
    cfg.update(kw)
    return cfg


def sp_np(t):
    t = t.coalesce()
    return t.indices().numpy().astype(np.int64), t.values().numpy().astype(np.float32)


def main():
    manifest = {}
    torch.set_num_threads(4)
    for cname, (nu, ni, spec) in CASES.items():
        edges = toy_edges() if spec is None else make_edges(spec[0], nu, ni, spec[1], spec[2])
        ds = ToyDataset(nu, ni, edges, name=cname)
        fx = {'n_users': np.int64(nu), 'n_items': np.int64(ni), 'train_array': edges.astype(np.int64)}

        # --- adjacency, degree, sym-normalised values (utils.py:42-50, model.py:89-98)
        adj = ref_utils.generate_daj_mat(ds)
        fx['adj_indptr'] = adj.indptr.astype(np.int64)
        fx['adj_indices'] = adj.indices.astype(np.int64)
        fx['adj_data'] = adj.data.astype(np.float32)
        deg = np.array(np.sum(adj, axis=1)).squeeze()
        fx['degree'] = deg.astype(np.float32)
        fx['dinv'] = np.power(np.maximum(1., deg), -0.5).astype(np.float32)

        torch.manual_seed(0)
        lg_cfg = model_cfg('LightGCN', ds, 32, 1)
        lg = ref_model.LightGCN(lg_cfg)
        idx, val = sp_np(lg.norm_adj)
        fx['norm_idx'] = idx
        fx['norm_val'] = val

        # --- LightGCN get_rep (model.py:100-110) at (d, L) in {(32,1), (64,2)}, + gradient
        for d, L in [(32, 1), (64, 2)]:
            torch.manual_seed(100 + d + L)
            m = ref_model.LightGCN(model_cfg('LightGCN', ds, d, L))
            m.eval()
            with torch.no_grad():
                rep = m.get_rep()
            fx[f'lgcn_d{d}_L{L}_emb'] = m.embedding.weight.detach().numpy().copy()
            fx[f'lgcn_d{d}_L{L}_rep'] = rep.numpy().copy()
            R = torch.randn(rep.shape, generator=torch.Generator().manual_seed(8))
            (m.get_rep() * R).sum().backward()
            fx[f'lgcn_d{d}_L{L}_R'] = R.numpy()
            fx[f'lgcn_d{d}_L{L}_grad'] = m.embedding.weight.grad.numpy().copy()

        # --- NGCF (model.py:3986-4055), eval mode: SpMM + 2 Linear + LeakyReLU + normalize, concat
        torch.manual_seed(500)
        m = ref_model.NGCF({'name': 'NGCF', 'embedding_size': 32, 'layer_sizes': [32, 32], 'device': 'cpu',
                            'dropout': 0.1, 'dataset': ds})
        m.eval()
        ni_, nv_ = sp_np(m.norm_adj)
        fx['ngcf_norm_idx'], fx['ngcf_norm_val'] = ni_, nv_
        fx['ngcf_emb'] = m.embedding.weight.detach().numpy().copy()
        for li in range(2):
            for nm, lay in [('gc', m.gc_layers[li]), ('bi', m.bi_layers[li])]:
                fx[f'ngcf_{nm}{li}_w'] = lay.weight.detach().numpy().copy()
                fx[f'ngcf_{nm}{li}_b'] = lay.bias.detach().numpy().copy()
        rep = m.get_rep()
        fx['ngcf_rep'] = rep.detach().numpy().copy()
        R = torch.randn(rep.shape, generator=torch.Generator().manual_seed(9))
        (rep * R).sum().backward()
        fx['ngcf_R'] = R.numpy()
        fx['ngcf_grad'] = m.embedding.weight.grad.numpy().copy()
        fx['ngcf_gc0_wgrad'] = m.gc_layers[0].weight.grad.numpy().copy()

        # --- IGCN: feat_mat (model.py:4139-4175), alpha anneal (4127-4134), get_rep (4188-4200)
        for d, L in [(64, 2), (32, 3)]:
            torch.manual_seed(200 + d + L)
            m = ref_model.IGCN(model_cfg('IGCN', ds, d, L))
            key = f'igcn_d{d}_L{L}'
            if d == 64:
                fi, fv = sp_np(m.feat_mat)
                fx['feat_idx'] = fi
                fx['feat_shape'] = np.array(m.feat_mat.shape, dtype=np.int64)
                fx['feat_val_a1'] = fv
                fx['row_sum'] = m.row_sum.numpy().copy()
            m.eval()
            emb = m.embedding.weight.detach().numpy().copy()
            with torch.no_grad():
                rep = m.get_rep()
            fx[key + '_emb'] = emb
            fx[key + '_rep'] = rep.numpy().copy()
            # gradient of sum(rep * R) w.r.t. the embedding table (gspmm backward)
            R = torch.randn(rep.shape, generator=torch.Generator().manual_seed(7))
            m.embedding.weight.grad = None
            (m.get_rep() * R).sum().backward()
            fx[key + '_R'] = R.numpy()
            fx[key + '_grad'] = m.embedding.weight.grad.numpy().copy()
            # dropout in train mode (model.py:4016-4028): rand drawn from the CPU generator
            m.train()
            torch.manual_seed(31)
            with torch.no_grad():
                rep_tr = m.get_rep()
            torch.manual_seed(31)
            fx[key + '_train_rand'] = torch.rand(m.feat_mat._nnz()).numpy()
            fx[key + '_train_rep'] = rep_tr.numpy().copy()
            m.eval()
            # BPR forward (model.py:4046-4052) and IGCNTrainer loss terms (trainer.py:535-551)
            g = np.random.RandomState(5)
            users = torch.tensor(g.randint(0, nu, size=16), dtype=torch.int64)
            pos = torch.tensor(g.randint(0, ni, size=16), dtype=torch.int64)
            neg = torch.tensor(g.randint(0, ni, size=16), dtype=torch.int64)
            with torch.no_grad():
                ur, pr, nr, l2 = m.bpr_forward(users, pos, neg)
                pos_s = torch.sum(ur * pr, dim=1)
                neg_s = torch.sum(ur * nr, dim=1)
                bpr = torch.nn.functional.softplus(neg_s - pos_s).mean()
                ue = m.embedding(users)
                pe = m.embedding(pos + len(m.user_map))
                ne = m.embedding(neg + len(m.user_map))
                aux = torch.nn.functional.softplus(torch.sum(ue * ne * m.w[None, :], dim=1)
                                                   - torch.sum(ue * pe * m.w[None, :], dim=1)).mean()
            fx[key + '_bpr_users'] = users.numpy()
            fx[key + '_bpr_pos'] = pos.numpy()
            fx[key + '_bpr_neg'] = neg.numpy()
            fx[key + '_bpr_l2'] = l2.numpy()
            fx[key + '_bpr_loss'] = np.float32(bpr.item())
            fx[key + '_aux_loss'] = np.float32(aux.item())
            if d == 64:
                for tag, n_anneal in [('a099sq', 2), ('a0', None)]:
                    if n_anneal is None:
                        m.alpha = 0.
                        m.update_feat_mat()
                    else:
                        m.alpha = 1.
                        for _ in range(n_anneal):
                            m.feat_mat_anneal()
                    fx[f'feat_val_{tag}'] = sp_np(m.feat_mat)[1]
                    fx[f'feat_alpha_{tag}'] = np.float64(m.alpha)

        # --- IMF (model.py:4290-4297): inductive layer only
        torch.manual_seed(300)
        m = ref_model.IMF(model_cfg('IMF', ds, 64, 0, dropout=0.1))
        m.eval()
        with torch.no_grad():
            fx['imf_emb'] = m.embedding.weight.detach().numpy().copy()
            fx['imf_rep'] = m.get_rep().numpy().copy()

        # --- AttIGCN (dead code, model.py:4223-4287): SDDMM + edge softmax + weighted SpMM
        AttIGCN = load_attigcn()
        torch.manual_seed(400)
        m = AttIGCN(model_cfg('AttIGCN', ds, 32, 2))
        m.eval()
        with torch.no_grad():
            fx['att_emb'] = m.embedding.weight.detach().numpy().copy()
            fx['att_wq'] = m.weight_q.weight.detach().numpy().copy()
            fx['att_bq'] = m.weight_q.bias.detach().numpy().copy()
            fx['att_wk'] = m.weight_k.weight.detach().numpy().copy()
            fx['att_bk'] = m.weight_k.bias.detach().numpy().copy()
            fx['att_feat_val'] = sp_np(m.feat_mat)[1]
            fx['att_alpha'] = m.inductive_rep_layer(m.feat_mat, return_alpha=True).numpy().copy()
            fx['att_x0'] = m.inductive_rep_layer(m.feat_mat).numpy().copy()
            fx['att_rep'] = m.get_rep().numpy().copy()
            # train mode: dropout REMOVES edges before the softmax (model.py:4016-4028, 4265-4274)
            m.train()
            torch.manual_seed(33)
            fx['att_train_rep'] = m.get_rep().numpy().copy()
            m.eval()

        # --- eval + calculate_metrics (trainer.py:115-210) on the d=64 IGCN
        torch.manual_seed(200 + 64 + 2)
        m = ref_model.IGCN(model_cfg('IGCN', ds, 64, 2))
        topks = [1, 5, 10, 20]
        kmax = min(20, ni)
        topks = [k for k in topks if k <= kmax]
        tcfg = {'name': 'BasicTrainer', 'dataset': ds, 'model': m, 'topks': topks, 'device': 'cpu',
                'n_epochs': 0, 'test_batch_size': 64}
        tr = ref_trainer.BasicTrainer(tcfg)
        for split in ['train', 'val', 'test']:
            _, metrics, _ = tr.eval(split)
            for mk in ['Precision', 'Recall', 'NDCG']:
                fx[f'eval_{split}_{mk}'] = np.array([metrics[mk][k] for k in topks], dtype=np.float64)
        fx['eval_topks'] = np.array(topks, dtype=np.int64)
        fx['eval_emb'] = m.embedding.weight.detach().numpy().copy()
        for split in ['val', 'test']:
            data = getattr(ds, split + '_data')
            fx[f'{split}_ptr'] = np.cumsum([0] + [len(x) for x in data]).astype(np.int64)
            fx[f'{split}_items'] = np.array(sum(data, []), dtype=np.int64)

        # calculate_metrics on fixed rec_items (synthetic ranking with ties to eval sets)
        g = np.random.RandomState(9)
        rec = np.stack([g.permutation(ni)[:kmax] for _ in range(nu)]).astype(np.int64)
        met = ref_trainer.BasicTrainer.calculate_metrics(types.SimpleNamespace(topks=topks), ds.test_data, rec)
        fx['cm_rec_items'] = rec
        for mk in ['Precision', 'Recall', 'NDCG']:
            fx[f'cm_{mk}'] = np.array([met[mk][k] for k in topks], dtype=np.float64)

        path = os.path.join(OUT, f'{cname}.npz')
        np.savez_compressed(path, **fx)
        manifest[cname] = {'n_users': nu, 'n_items': ni, 'n_train': int(len(edges)),
                           'nnz_adj': int(len(fx['norm_val'])), 'nnz_feat': int(len(fx['feat_val_a1'])),
                           'bytes': os.path.getsize(path)}
        print(cname, manifest[cname])

    # --- raw ingestion: the reference's GowallaDataset (dataset.py:167-189) on a synthetic
    # check-in file -> remove_sparse_ui + update_user_inter_lists + generate_data (dataset.py:66-114)
    import tempfile
    sys.path.insert(0, OUT)
    import ml_like
    import dataset as ref_dataset
    os.environ['TZ'] = 'UTC'
    import time as _time
    _time.tzset()
    with tempfile.TemporaryDirectory() as tmp:
        ml_like.write_checkins(os.path.join(tmp, 'Gowalla_totalCheckins.txt'))
        ig = {}
        for tag, mi in [('k5', 5), ('k10', 10)]:
            ds = ref_dataset.GowallaDataset({'name': 'GowallaDataset', 'path': tmp, 'device': 'cpu',
                                             'min_inter': mi, 'split_ratio': [0.8, 0.1, 0.1]})
            ig[f'{tag}_n'] = np.array([ds.n_users, ds.n_items], np.int64)
            for split in ['train', 'val', 'test']:
                data = getattr(ds, split + '_data')
                ig[f'{tag}_{split}_ptr'] = np.cumsum([0] + [len(x) for x in data]).astype(np.int64)
                ig[f'{tag}_{split}_items'] = np.array(sum(data, []), dtype=np.int64)
        np.savez_compressed(os.path.join(OUT, 'ingest_gowalla.npz'), **ig)
        print('ingest', {k: v.tolist() for k, v in ig.items() if k.endswith('_n')})

    manifest['_generator'] = {
        'reference': 'umaDosey/Inductive-Recommendation @ /root/reference (v1)',
        'torch': torch.__version__, 'numpy': np.__version__,
        'stubs': 'dgl (gspmm restated from DGL docs), info_nce, torchmetrics.functional',
    }
    with open(os.path.join(OUT, 'manifest.json'), 'w') as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
