"""igr.model - the reference's model surface on the MI355X path.

Same class names, constructor config dicts and methods as the reference's
model.py (get_model, BasicModel.predict/save/load, LightGCN, NGCF, IGCN, IMF,
and the AttIGCN that the reference keeps as dead text at model.py:4223-4287),
so the reference's trainers and configs drive them unchanged.  The graph
structure is built once in __init__ (C++ host builder) and lives in HBM;
every propagation runs through the HIP kernels (igr.ops).
"""
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.init import kaiming_uniform_, normal_, zeros_

from . import ops
from .graph import Graph, csr_from_coo, row_sums, sym_norm_values


def get_model(config, dataset):
    """model.py:20-25."""
    config = config.copy()
    config['dataset'] = dataset
    model = getattr(sys.modules[__name__], config['name'])
    return model(config)


def init_one_layer(in_features, out_features):
    """model.py:28-32."""
    layer = nn.Linear(in_features, out_features)
    kaiming_uniform_(layer.weight)
    zeros_(layer.bias)
    return layer


def train_pairs(dataset):
    """dataset.train_array as an int64 [E, 2] array (reference: list of [u, i])."""
    ta = getattr(dataset, 'train_pairs', None)
    if ta is None:
        ta = np.asarray(dataset.train_array, dtype=np.int64).reshape(-1, 2)
    return ta


def build_norm_adj(n_users, n_items, pairs, device):
    """utils.generate_daj_mat (utils.py:42-50) + LightGCN.generate_graph (model.py:89-98).

    Returns (Graph marked symmetric, values float32 tensor, degree, dinv).
    degree = fp32 row sum (duplicates count twice, as scipy sums them);
    dinv = np.power(max(1, degree), -0.5) in float32 on the host - the same
    numpy call the reference makes (its SIMD pow is host-ISA dependent, so it
    is not recomputed on the device); value = (dinv_r * a) * dinv_c."""
    u, i = pairs[:, 0], pairs[:, 1]
    n = n_users + n_items
    row = np.concatenate([u, i + n_users])
    col = np.concatenate([i + n_users, u])
    rp, ci, v, _ = csr_from_coo(row, col, n, n, None, dedup=True, want_eid=False)
    degree = row_sums(rp, v)
    dinv = np.power(np.maximum(np.float32(1.), degree), np.float32(-0.5)).astype(np.float32)
    vals = sym_norm_values(rp, ci, v, dinv)
    g = Graph(rp, ci, n, n, device=device, symmetric=True)
    return g, torch.from_numpy(vals).to(device), degree, dinv


def batch_edges_estimate(row_ptr, col_idx, n_users, batch_size):
    """Expected adjacency edges the 3B rows of a BPR batch touch, under the
    trainers' sampling: a uniform active user, a uniform item of that user, a
    uniform item (sampler.py / dataset.BPRBatchSampler)."""
    deg = np.diff(row_ptr).astype(np.float64)
    ud = deg[:n_users]
    active = np.nonzero(ud > 0)[0]
    if len(active) == 0:
        return 0.0
    pos = np.add.reduceat(deg[col_idx[:row_ptr[n_users]]], row_ptr[:n_users][active]) / ud[active]
    item = deg[n_users:].mean() if len(deg) > n_users else 0.0
    return float(batch_size * (ud[active].mean() + pos.mean() + item))


def batch_rep_pays(model, batch_size):
    """Whether a BPR step should compute the last propagation layer only at the
    batch rows (ops.propagate_rows) instead of over the whole graph.

    model.config['batch_rep']: True / False, or 'auto' (default): take the row
    path when the batch rows touch fewer than a quarter of the graph's edges
    (batch_edges_estimate; the restricted forward + atomic push cost ~3-4x a
    streamed edge)."""
    mode = model.config.get('batch_rep', 'auto')
    if mode != 'auto':
        return bool(mode)
    cache = model.__dict__.setdefault('_batch_rep_cache', {})
    if batch_size not in cache:
        h = model.norm_adj.host()
        est = batch_edges_estimate(h['row_ptr'], h['col_idx'], model.n_users, batch_size)
        cache[batch_size] = bool(4 * est < model.norm_adj.nnz)
    return cache[batch_size]


def load_checkpoint(path, device):
    """torch.load that executes nothing from the file (weights_only), widened by
    the three numpy names a pickled numpy integer scalar refers to - the keys of
    the user_map / item_map dicts in a checkpoint IGCN.save of the reference
    wrote (model.py:4208-4211: the maps are built from np.arange, 4147-4156)."""
    import numpy.dtypes
    try:
        from numpy._core.multiarray import scalar
    except ImportError:  # numpy < 2
        from numpy.core.multiarray import scalar
    with torch.serialization.safe_globals([scalar, np.dtype, numpy.dtypes.Int64DType]):
        return torch.load(path, map_location=device, weights_only=True)


class BasicModel(nn.Module):
    """model.py:35-53."""

    def __init__(self, model_config):
        super().__init__()
        self.config = model_config
        self.name = model_config['name']
        self.device = model_config['device']
        self.n_users = model_config['dataset'].n_users
        self.n_items = model_config['dataset'].n_items
        self.trainable = True

    @property
    def graph_safe(self):
        """May a training step of this model be captured in a hipGraph and replayed with the
        same results as eager steps?  Yes when nothing in the step is drawn on the host or from
        torch's generator: dropout masks from device counters (IGCN family, unless
        dropout_rng = 'cpu'), or no dropout at all."""
        if not torch.device(self.device).type == 'cuda':
            return False
        if isinstance(self, (IGCN, LightGCN)):
            return self.config.get('dropout_rng', 'device') != 'cpu' or getattr(self, 'dropout', 0) == 0
        return isinstance(self, (NGCF, IMCGAE)) and getattr(self, 'dropout', 0) == 0

    @property
    def norm_vals(self):
        """The adjacency's edge values by edge id (the reference keeps them inside
        its sparse norm_adj; here they ride on the Graph generate_graph returns)."""
        return self.norm_adj.values

    def predict(self, users):
        raise NotImplementedError

    def _join_batch_stream(self, *tensors):
        """A caller that drew the batch on another stream (trainer.StepGraph: the sampling then
        runs beside the propagation, which does not read it) leaves that stream in
        `_batch_stream`; the current stream waits for it here, just before the batch's first use."""
        bs = self.__dict__.pop('_batch_stream', None)
        if bs is not None:
            cur = torch.cuda.current_stream()
            cur.wait_stream(bs)
            for t in tensors:
                t.record_stream(cur)

    def save(self, path):
        torch.save(self.state_dict(), path)

    def load(self, path):
        self.load_state_dict(load_checkpoint(path, self.device))


class LightGCN(BasicModel):
    """model.py:79-127: rep = mean_l A^l E over the symmetric-normalised bipartite graph."""

    def __init__(self, model_config):
        super().__init__(model_config)
        self.embedding_size = model_config['embedding_size']
        self.n_layers = model_config['n_layers']
        self.embedding = nn.Embedding(self.n_users + self.n_items, self.embedding_size)
        self.norm_adj = self.generate_graph(model_config['dataset'])
        normal_(self.embedding.weight, std=0.1)
        self.to(device=self.device)

    def generate_graph(self, dataset):
        """model.py:89-98: one object, as the reference's sparse norm_adj - the
        Graph with its edge values attached (`.values`, what `norm_vals` reads)."""
        g, vals, self.degree, self.dinv = build_norm_adj(self.n_users, self.n_items, train_pairs(dataset),
                                                         self.device)
        g.values = vals
        return g

    def get_rep(self):
        """model.py:100-110, fused (one SpMM per layer, running layer mean)."""
        return ops.propagate(self.norm_adj, self.embedding.weight, self.n_layers, adj_vals=self.norm_vals)

    def bpr_forward(self, users, pos_items, neg_items):
        rep = self.get_rep()
        e = self.embedding.weight
        users_e = ops.gather(e, users)
        pos_e, neg_e = ops.gather(e, pos_items, self.n_users), ops.gather(e, neg_items, self.n_users)
        l2_norm_sq = (users_e ** 2).sum(1) + (pos_e ** 2).sum(1) + (neg_e ** 2).sum(1)
        users_r = ops.gather(rep, users)
        pos_r, neg_r = ops.gather(rep, pos_items, self.n_users), ops.gather(rep, neg_items, self.n_users)
        return users_r, pos_r, neg_r, l2_norm_sq

    def predict(self, users, rep=None):
        rep = self.get_rep() if rep is None else rep
        users_r = ops.gather(rep, users)
        return ops.gemm(users_r, rep[self.n_users:])

    def bpr_loss(self, users, pos_items, neg_items, need_l2=True):
        """Fused LightGCN/BPRTrainer step terms: (bpr loss, mean l2 of raw embeddings).
        The last layer runs only at the batch rows when batch_rep_pays.  need_l2=False
        (a trainer whose l2_reg is 0: the term and its gradient are exact zeros) skips
        the l2 pass and returns None for it."""
        if batch_rep_pays(self, users.numel()):
            self._join_batch_stream(users, pos_items, neg_items)
            rows, (iu, ip, ineg) = ops.batch_rows(users, pos_items, neg_items, self.n_users)
            rep_b = ops.propagate_rows(self.norm_adj, self.embedding.weight, self.n_layers, rows,
                                       adj_vals=self.norm_vals)
            bpr, _ = ops.bpr_loss(rep_b, iu, ip, ineg, 0, 0, distinct=True)
            keys = None
        else:
            rep = self.get_rep()
            self._join_batch_stream(users, pos_items, neg_items)
            # both terms scatter their gradients over the same table rows: one sort serves both
            keys = ops.rowsort(users, 0, pos_items, self.n_users, neg_items, self.n_users) \
                if need_l2 and torch.is_grad_enabled() else None
            bpr, _ = ops.bpr_loss(rep, users, pos_items, neg_items, 0, self.n_users, keys=keys)
        if not need_l2:
            return bpr, None
        _, l2 = ops.bpr_loss(self.embedding.weight, users, pos_items, neg_items, 0, self.n_users, keys=keys)
        return bpr, l2


class NGCF(BasicModel):
    """model.py:3986-4055 (dense d x d layers on the MFMA GEMM)."""

    def __init__(self, model_config):
        super().__init__(model_config)
        self.dropout = model_config['dropout']
        self.embedding_size = model_config['embedding_size']
        self.layer_sizes = model_config['layer_sizes'].copy()
        self.embedding = nn.Embedding(self.n_users + self.n_items, self.embedding_size)
        kaiming_uniform_(self.embedding.weight)
        self.n_layers = len(self.layer_sizes)
        self.layer_sizes.insert(0, self.embedding_size)
        # layer by layer, the gc layer before the bi layer: the generator's draws land on the same
        # weights as in the reference's constructor (model.py:3998-4002)
        gc, bi = [], []
        for i in range(1, self.n_layers + 1):
            gc.append(init_one_layer(self.layer_sizes[i - 1], self.layer_sizes[i]))
            bi.append(init_one_layer(self.layer_sizes[i - 1], self.layer_sizes[i]))
        self.gc_layers, self.bi_layers = nn.ModuleList(gc), nn.ModuleList(bi)
        self.norm_adj = self.generate_graph(model_config['dataset'])
        self.to(device=self.device)

    def generate_graph(self, dataset):
        """adj + I, row-normalised (sklearn normalize l1, model.py:4009-4014)."""
        pairs = train_pairs(dataset)
        n = self.n_users + self.n_items
        u, i = pairs[:, 0], pairs[:, 1]
        row = np.concatenate([u, i + self.n_users, np.arange(n)])
        col = np.concatenate([i + self.n_users, u, np.arange(n)])
        rp, ci, v, _ = csr_from_coo(row, col, n, n, None, dedup=True, want_eid=False)
        rs = row_sums(rp, v)
        vals = (v / np.repeat(rs, np.diff(rp))).astype(np.float32)
        g = Graph(rp, ci, n, n, device=self.device)
        g.values = torch.from_numpy(vals).to(self.device)
        return g

    def dropout_values(self, vals):
        return dropout_values(self, vals)

    def dropout_sp_mat(self, mat):
        """model.py:4016-4028, same call: `mat` a graph carrying edge values (norm_adj,
        or the feat_mat of an IGCN passed as self, as at model.py:4189); returns that
        graph with the dropped values (a view, Graph.with_values).  The fused paths
        (get_rep) draw the same masks without materialising this."""
        counter = mat if hasattr(self, 'next_dropout_step') else None  # IGCN: the fused path's draws
        return mat.with_values(dropout_values(self, graph_values(self, mat), counter))

    def get_rep(self):
        representations = self.embedding.weight
        all_layer_rep = [representations]
        vals = self.dropout_values(self.norm_vals)
        for layer_idx in range(self.n_layers):
            m0 = ops.gspmm(self.norm_adj, 'mul', 'sum', representations, vals)
            m1 = representations * m0
            m0 = ops.linear(m0, self.gc_layers[layer_idx])
            m1 = ops.linear(m1, self.bi_layers[layer_idx])
            if m0.shape[1] <= ops.LAYER_TAIL_MAX_WIDTH:  # activation, dropout and row norm in one kernel
                representations, normed = ops.layer_tail(m0, m1, self.dropout, self.training, slope=0.2)
            else:
                representations = F.leaky_relu(m0 + m1, negative_slope=0.2)
                representations = F.dropout(representations, p=self.dropout, training=self.training)
                normed = F.normalize(representations, p=2, dim=1)
            all_layer_rep.append(normed)
        return torch.cat(all_layer_rep, dim=1)

    def bpr_forward(self, users, pos_items, neg_items):
        """model.py:4046-4052: gathers from rep; l2 over the gathered rep rows."""
        rep = self.get_rep()
        users_r = ops.gather(rep, users)
        pos_r, neg_r = ops.gather(rep, pos_items, self.n_users), ops.gather(rep, neg_items, self.n_users)
        l2_norm_sq = (users_r ** 2).sum(1) + (pos_r ** 2).sum(1) + (neg_r ** 2).sum(1)
        return users_r, pos_r, neg_r, l2_norm_sq

    def bpr_loss(self, users, pos_items, neg_items, need_l2=True):
        """Fused BPRTrainer step terms (trainer.py:410-421 over model.py:4046-4052): (bpr loss,
        mean l2 of the gathered rep rows) from one pass over the batch's rep rows."""
        rep = self.get_rep()
        self._join_batch_stream(users, pos_items, neg_items)
        bpr, l2 = ops.bpr_loss(rep, users, pos_items, neg_items, 0, self.n_users)
        return bpr, (l2 if need_l2 else None)

    def predict(self, users, rep=None):
        return LightGCN.predict(self, users, rep)


def graph_values(model, mat):
    """The edge values of `mat` by edge id: the ones it carries, or the model's
    feature values when it is the model's feature graph."""
    if mat.values is not None:
        return mat.values
    if mat is getattr(model, 'feat_mat', None):
        return model.feat_vals
    raise ValueError('this graph carries no edge values')


def dropout_values(model, vals, graph=None):
    """NGCF.dropout_sp_mat (model.py:4016-4028) as a value mask over the fixed
    CSR (a dropped edge contributes an exact 0.0).  config['dropout_rng'] =
    'cpu' draws the uniforms from the CPU generator exactly as the reference
    does (`torch.rand(nnz).to(device)`), for run-to-run parity with it; a graph
    given with the default 'device' draws them from the counter-based device
    generator keyed by (seed, step, edge) - the draws of the fused-dropout SpMM,
    the same in eager steps and in hipGraph replays."""
    if not model.training or model.dropout == 0:
        return vals
    n = vals.numel()
    if model.config.get('dropout_rng', 'device') == 'cpu':
        rand = torch.rand(n).to(vals.device)
    elif graph is not None:
        seed, step, ctr = model.next_dropout_step()
        return ops.edge_dropout_counter(graph, vals, model.dropout, seed, step, offset_dev=ctr)
    else:
        rand = torch.rand(n, device=vals.device)
    return ops.edge_dropout(vals, rand, model.dropout)


class IGCN(BasicModel):
    """model.py:4107-4220: template-feature inductive layer + LightGCN layers."""

    def __init__(self, model_config):
        super().__init__(model_config)
        self.embedding_size = model_config['embedding_size']
        self.n_layers = model_config['n_layers']
        self.dropout = model_config['dropout']
        self.feature_ratio = model_config['feature_ratio']
        self.norm_adj = self.generate_graph(model_config['dataset'])
        self.alpha = 1.
        self.delta = model_config.get('delta', 0.99)
        self.feat_mat, self.user_map, self.item_map, self.row_sum = \
            self.generate_feat(model_config['dataset'], ranking_metric=model_config.get('ranking_metric', 'sort'))
        self.update_feat_mat()
        self.embedding = nn.Embedding(self.feat_mat.n_cols, self.embedding_size)
        self.w = nn.Parameter(torch.ones([self.embedding_size], dtype=torch.float32, device=self.device))
        normal_(self.embedding.weight, std=0.1)
        self.to(device=self.device)

    def generate_graph(self, dataset):
        """model.py:89-98: one object, as the reference's sparse norm_adj - the
        Graph with its edge values attached (`.values`, what `norm_vals` reads)."""
        g, vals, self.degree, self.dinv = build_norm_adj(self.n_users, self.n_items, train_pairs(dataset),
                                                         self.device)
        g.values = vals
        return g

    def update_feat_mat(self):
        """model.py:4127-4130: value = row_sum[row] ** ((alpha - 1)/2 - 0.5), on the device.
        The value is row-constant, so one value per row (feat_base) is kept; the
        per-edge array (feat_vals) is materialised only when asked for."""
        ex = (self.alpha - 1.) / 2. - 0.5
        # in place once allocated: a captured training step (trainer.StepGraph) holds these pointers.
        # A feature graph regenerated for another dataset (generate_feat(..., is_updating=True) after
        # new users / items arrived, model.py:4219) has other sizes: its buffers start afresh.
        base = getattr(self, 'feat_base', None)
        if base is not None and base.numel() != self.row_sum.numel():
            base = None
        fv = getattr(self, '_feat_vals', None)
        if fv is not None and fv.numel() != self.feat_mat.nnz:
            fv = self._feat_vals = None
        self.feat_base = ops.feat_row_values(self.row_sum, ex, out=base)
        if fv is not None:
            ops.feat_values(self.feat_mat, self.row_sum, ex, out=fv)

    @property
    def feat_vals(self):
        """Per-edge feature values (by edge id), as the reference's feat_mat.values()."""
        if getattr(self, '_feat_vals', None) is None:
            ex = (self.alpha - 1.) / 2. - 0.5
            self._feat_vals = ops.feat_values(self.feat_mat, self.row_sum, ex)
        return self._feat_vals

    def feat_mat_anneal(self):
        """model.py:4132-4134."""
        self.alpha *= self.delta
        self.update_feat_mat()

    def generate_feat(self, dataset, is_updating=False, ranking_metric=None):
        """model.py:4139-4175, vectorised: user u -> feature U' + item_map[i],
        item i -> user_map[u], plus one 'general' feature per side; the COO
        goes through the same duplicate-summing CSR build."""
        if not is_updating:
            if self.feature_ratio < 1.:
                ranked_users, ranked_items = graph_rank_nodes(dataset, ranking_metric)
                core_users = ranked_users[:int(self.n_users * self.feature_ratio)]
                core_items = ranked_items[:int(self.n_items * self.feature_ratio)]
            else:
                core_users = np.arange(self.n_users, dtype=np.int64)
                core_items = np.arange(self.n_items, dtype=np.int64)
            user_map = {int(u): k for k, u in enumerate(core_users)}
            item_map = {int(i): k for k, i in enumerate(core_items)}
        else:
            user_map, item_map = self.user_map, self.item_map
        umap = np.full(self.n_users, -1, np.int64)
        imap = np.full(self.n_items, -1, np.int64)
        if user_map:
            umap[np.fromiter(user_map.keys(), np.int64)] = np.fromiter(user_map.values(), np.int64)
        if item_map:
            imap[np.fromiter(item_map.keys(), np.int64)] = np.fromiter(item_map.values(), np.int64)
        user_dim, item_dim = len(user_map), len(item_map)
        pairs = train_pairs(dataset)
        u, i = pairs[:, 0], pairs[:, 1]
        ki, ku = imap[i] >= 0, umap[u] >= 0
        U, I = self.n_users, self.n_items
        row = np.concatenate([u[ki], U + i[ku], np.arange(U), U + np.arange(I)])
        col = np.concatenate([user_dim + imap[i[ki]], umap[u[ku]], np.full(U, user_dim + item_dim),
                              np.full(I, user_dim + item_dim + 1)])
        n_cols = user_dim + item_dim + 2
        rp, ci, v, _ = csr_from_coo(row, col, U + I, n_cols, None, dedup=True, want_eid=False)
        row_sum = torch.from_numpy(row_sums(rp, v)).to(self.device)
        feat = Graph(rp, ci, U + I, n_cols, device=self.device)
        return feat, user_map, item_map, row_sum

    def feat_values(self):
        """Feature-graph weights for one get_rep (dropout_sp_mat, model.py:4189).

        Default: ScaledWeights - row-constant values with the dropout mask drawn
        inside the SpMM from a counter-based RNG (no rand tensor, no value
        array; the backward regenerates the same mask).  dropout_rng = 'cpu'
        instead materialises the values with the reference's own CPU-generator
        draws (bit-for-bit the reference's mask)."""
        if self.training and self.dropout > 0 and self.config.get('dropout_rng', 'device') == 'cpu':
            return dropout_values(self, self.feat_vals)
        if self.training and self.dropout > 0:
            seed, step, ctr = self.next_dropout_step()
            return ops.ScaledWeights(self.feat_base, None, 1.0 - self.dropout, seed, step, offset_dev=ctr)
        return ops.ScaledWeights(self.feat_base)

    def next_dropout_step(self):
        """(seed, offset, device counter or None) of this step's dropout draws.  Eager:
        the host step count, advanced here.  hipGraph mode (device_step set): the
        next host step plus the replays so far, which the kernels add on the device."""
        if not hasattr(self, '_drop_seed'):
            self._drop_seed = int(self.config.get('seed', torch.initial_seed())) & (2 ** 63 - 1)
        ctr = getattr(self, 'device_step', None)
        if ctr is not None:
            return self._drop_seed, getattr(self, '_drop_step', -1) + 1, ctr
        self._drop_step = getattr(self, '_drop_step', -1) + 1
        return self._drop_seed, self._drop_step, None

    def inductive_rep_layer(self, feat_vals):
        """model.py:4177-4186 (no padding needed: the lhs has n_cols rows).  Takes the
        reference's argument - the feature graph with its (dropped) values - or the
        values alone."""
        if isinstance(feat_vals, Graph):
            feat_vals = graph_values(self, feat_vals)
        if isinstance(feat_vals, ops.ScaledWeights):
            return ops.propagate(self.norm_adj, self.embedding.weight, 0, feat=self.feat_mat, fvals=feat_vals)
        return ops.gspmm(self.feat_mat, 'mul', 'sum', self.embedding.weight, feat_vals)

    def inductive_values(self):
        """Weights of the inductive layer for one get_rep (dropout applied in training)."""
        return self.feat_values()

    def get_rep(self):
        """model.py:4188-4200, fused: inductive SpMM + L layers + layer mean."""
        return ops.propagate(self.norm_adj, self.embedding.weight, self.n_layers, feat=self.feat_mat,
                             fvals=self.inductive_values(), adj_vals=self.norm_vals)

    def bpr_forward(self, users, pos_items, neg_items):
        return NGCF.bpr_forward(self, users, pos_items, neg_items)

    def predict(self, users, rep=None):
        return LightGCN.predict(self, users, rep)

    def _rows_path(self, batch_size):
        return self.n_layers > 0 and batch_rep_pays(self, batch_size)

    def _l2_extra(self):
        return None

    def bpr_loss(self, users, pos_items, neg_items, need_l2=True):
        """Fused IGCNTrainer terms on rep: (bpr loss, mean l2 of rep rows).
        The last layer runs only at the batch rows when batch_rep_pays.  need_l2=False
        (l2_reg = 0, as in the reference's IGCN configs: the term and its gradient are
        exact zeros) returns None for l2 and skips AttIGCN's projection norms."""
        if self._rows_path(users.numel()):
            self._join_batch_stream(users, pos_items, neg_items)
            rows, (iu, ip, ineg) = ops.batch_rows(users, pos_items, neg_items, self.n_users)
            rep_b = ops.propagate_rows(self.norm_adj, self.embedding.weight, self.n_layers, rows,
                                       feat=self.feat_mat, fvals=self.inductive_values(), adj_vals=self.norm_vals)
            bpr, l2 = ops.bpr_loss(rep_b, iu, ip, ineg, 0, 0, distinct=True)
        else:
            rep = self.get_rep()
            self._join_batch_stream(users, pos_items, neg_items)
            keys = self.__dict__.pop('_bpr_keys', None)  # sorted on the aux stream (bpr_aux_loss)
            if keys is not None:
                cur = torch.cuda.current_stream()
                cur.wait_stream(self._aux_side)
                keys.record_stream(cur)
            bpr, l2 = ops.bpr_loss(rep, users, pos_items, neg_items, 0, self.n_users, keys=keys)
        if not need_l2:
            return bpr, None
        extra = self._l2_extra()
        return bpr, (l2 if extra is None else l2 + extra)

    def bpr_aux_loss(self, users, pos_items, neg_items, a_users, a_pos, a_neg, need_l2=True):
        """All three IGCNTrainer.step terms (trainer.py:536-549): (bpr, l2, aux).
        On the row path the aux term rides in the same autograd node, so its
        gradient is added into the embedding gradient in place."""
        if not self._rows_path(users.numel()):
            side = self._aux_stream()
            if side is None:
                bpr, l2 = self.bpr_loss(users, pos_items, neg_items, need_l2)
                return bpr, l2, self.aux_loss(a_users, a_pos, a_neg)
            # the aux term touches only the raw table: its forward (and, through autograd's stream
            # bookkeeping, its backward) runs on a second stream beside the propagation
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            drawn_on = getattr(self, '_batch_stream', None)  # the batches' stream, if not this one's
            if drawn_on is not None and drawn_on is not side:
                side.wait_stream(drawn_on)
            with torch.cuda.stream(side):
                for t in (a_users, a_pos, a_neg):
                    t.record_stream(side)
                if self.training and torch.is_grad_enabled():
                    # the sort the main term's backward walks depends on the batch alone: done here,
                    # beside the propagation, instead of between the loss and its gradient
                    for t in (users, pos_items, neg_items):
                        t.record_stream(side)
                    self._bpr_keys = ops.rowsort(users, 0, pos_items, self.n_users, neg_items, self.n_users)
                aux = self.aux_loss(a_users, a_pos, a_neg)
            try:
                bpr, l2 = self.bpr_loss(users, pos_items, neg_items, need_l2)
            finally:
                self.__dict__.pop('_bpr_keys', None)  # never left for a later, different batch
            cur.wait_stream(side)
            aux.record_stream(cur)
            return bpr, l2, aux
        self._join_batch_stream(users, pos_items, neg_items, a_users, a_pos, a_neg)
        rows, (iu, ip, ineg) = ops.batch_rows(users, pos_items, neg_items, self.n_users)
        rep_b, aux = ops.propagate_rows(self.norm_adj, self.embedding.weight, self.n_layers, rows,
                                        feat=self.feat_mat, fvals=self.inductive_values(), adj_vals=self.norm_vals,
                                        aux=(a_users, a_pos, a_neg, len(self.user_map)), w=self.w)
        bpr, l2 = ops.bpr_loss(rep_b, iu, ip, ineg, 0, 0, distinct=True)
        if not need_l2:
            return bpr, None, aux
        extra = self._l2_extra()
        return bpr, (l2 if extra is None else l2 + extra), aux

    def _aux_stream(self):
        """The stream of the aux term inside a hipGraph-captured step (config 'aux_stream': True
        forces it in eager steps too, False switches it off); default priority, as every stream
        here.  In a captured step the two branches become independent graph nodes; an eager step
        is bound by the host, which a second stream does not help."""
        want = self.config.get('aux_stream', 'capture')
        if want is False or not self.embedding.weight.is_cuda:
            return None
        if want == 'capture' and not torch.cuda.is_current_stream_capturing():
            return None
        if getattr(self, '_aux_side', None) is None:
            self._aux_side = torch.cuda.Stream(device=self.embedding.weight.device)
        return self._aux_side

    def backward_scope(self):
        """Context for loss.backward() of a step whose aux term ran on the side stream: the
        table's gradient then arrives from two streams by design (autograd orders them), and
        autograd's warning about that is switched off for the backward only and switched back
        on after it - not for the rest of the process."""
        import contextlib
        setter = getattr(torch.autograd.graph, 'set_warn_on_accumulate_grad_stream_mismatch', None)
        if getattr(self, '_aux_side', None) is None or setter is None:
            return contextlib.nullcontext()

        @contextlib.contextmanager
        def scope():
            setter(False)
            try:
                yield
            finally:
                setter(True)  # torch's default
        return scope()

    def aux_loss(self, users, pos_items, neg_items):
        """IGCNTrainer aux term (trainer.py:542-549) on the raw feature table with w."""
        loss, _ = ops.bpr_loss(self.embedding.weight, users, pos_items, neg_items, 0, len(self.user_map), w=self.w)
        return loss

    def save(self, path):
        """model.py:4208-4211 (key 'sate_dict' kept as in the reference)."""
        torch.save({'sate_dict': self.state_dict(), 'user_map': self.user_map, 'item_map': self.item_map,
                    'alpha': self.alpha}, path)

    def load(self, path):
        """model.py:4213-4220.  Reads this class's checkpoints and the reference's
        own (same keys; its user_map / item_map are keyed by numpy int64 scalars)
        with the restricted loader: tensors, numbers and dicts only."""
        params = load_checkpoint(path, self.device)
        self.load_state_dict(params['sate_dict'])
        self.user_map = {int(k): int(v) for k, v in params['user_map'].items()}
        self.item_map = {int(k): int(v) for k, v in params['item_map'].items()}
        self.alpha = float(params['alpha'])
        self.feat_mat, _, _, self.row_sum = self.generate_feat(self.config['dataset'], is_updating=True)
        self.update_feat_mat()


class IMF(IGCN):
    """model.py:4290-4297: the inductive layer alone."""

    def get_rep(self):
        return ops.propagate(self.norm_adj, self.embedding.weight, 0, feat=self.feat_mat,
                             fvals=self.feat_values(), adj_vals=self.norm_vals)

    def _rows_path(self, batch_size):
        return False  # the inductive layer alone: rep = F E


class AttIGCN(IGCN):
    """Attention inductive layer (dead text in the reference, model.py:4223-4287).

    x_k = Wk E;  x_q = Wq (F E);  alpha = SDDMM(x_q, x_k) over feat_mat;
    edge softmax with max-shift, exp(./sqrt(d)/10), head mean; out = SpMM(E, w).
    The reference detaches E inside the projections (model.py:4258, 4262)."""

    def __init__(self, model_config):
        BasicModel.__init__(self, model_config)
        self.embedding_size = model_config['embedding_size']
        self.n_layers = model_config['n_layers']
        self.n_heads = model_config.get('n_heads', 4)
        self.dropout = model_config['dropout']
        self.feature_ratio = 1.
        self.alpha = 0.
        self.delta = model_config.get('delta', 0.99)
        self.norm_adj = self.generate_graph(model_config['dataset'])
        self.feat_mat, self.user_map, self.item_map, self.row_sum = self.generate_feat(model_config['dataset'])
        self.update_feat_mat()
        self.embedding = nn.Embedding(self.feat_mat.n_cols, self.embedding_size)
        kaiming_uniform_(self.embedding.weight)
        self.weight_q = init_one_layer(self.embedding_size, self.embedding_size * self.n_heads)
        self.weight_k = init_one_layer(self.embedding_size, self.embedding_size * self.n_heads)
        self.w = nn.Parameter(torch.ones([self.embedding_size], dtype=torch.float32, device=self.device))
        self.to(device=self.device)

    def feat_values(self):
        """Explicit per-edge dropout values: the attention layer needs them per edge."""
        return dropout_values(self, self.feat_vals, self.feat_mat)

    def attention_values(self, feat_vals):
        """model.py:4258-4275.  After dropout the dropped edges are absent from
        the reference's graph; here they carry value 0 and are excluded from
        the softmax through `keep`.

        Default ('attention': 'folded'): the key projection is folded into the query
        side.  <x_q[r, j], W_k[j] E[c] + b_k[j]> = <W_k[j]^T x_q[r, j], E[c]> + a term
        constant over row r's edges, which the row softmax cancels exactly; and
        W_k[j]^T (W_q[j] y + b_q[j]) is again one Linear(d, h d) of y = F E, with
        weight M[j] = W_k[j]^T W_q[j] and bias W_k[j]^T b_q[j].  So x_k is never
        formed (one projection GEMM instead of two), every edge gathers the d floats
        of E[c] instead of the h d floats of x_k[c], and the backward has no
        reverse-graph per-head SpMM (b_k's gradient is the exact zero the reference's
        is up to rounding).  'attention': 'reference' keeps the reference's operation
        order (x_k formed, per-head gathers)."""
        e = self.embedding.weight.detach()
        y = ops.gspmm(self.feat_mat, 'mul', 'sum', e, feat_vals)
        keep = feat_vals if (self.training and self.dropout > 0) else None
        H, d = self.n_heads, self.embedding_size
        if self.config.get('attention', 'folded') == 'reference' or not self._foldable():
            x_k = ops.linear(e, self.weight_k)
            x_q = ops.linear(y, self.weight_q)
            alpha = ops.gsddmm(self.feat_mat, 'dot', x_q, x_k, h=H)
        else:
            wq, wk = self.weight_q.weight.view(H, d, d), self.weight_k.weight.view(H, d, d)
            m = torch.bmm(wk.transpose(1, 2), wq).reshape(H * d, d)                        # M[j] = W_k[j]^T W_q[j]
            b = torch.bmm(wk.transpose(1, 2), self.weight_q.bias.view(H, d, 1)).reshape(H * d)
            # b_k only shifts every edge of a row alike: no effect after the softmax, zero gradient
            b = b + 0. * self.weight_k.bias.sum()
            u = ops.Linear.apply(y, m, b)
            alpha = ops.GSDDMMShared.apply(self.feat_mat, u, e, H)
        return ops.AttSoftmax.apply(self.feat_mat, alpha, ops.sqrt_scale(self.embedding_size), keep)

    def _foldable(self):
        d, H = self.embedding_size, self.n_heads
        return d in (32, 64, 128, 256) and H in (1, 2, 4, 8) and H * d <= 512

    def inductive_rep_layer(self, feat_vals, return_alpha=False):
        if isinstance(feat_vals, Graph):
            feat_vals = graph_values(self, feat_vals)
        w = self.attention_values(feat_vals)
        if return_alpha:
            return w
        return ops.gspmm(self.feat_mat, 'mul', 'sum', self.embedding.weight, w)

    def inductive_values(self):
        return self.attention_values(self.feat_values())

    def _l2_extra(self):
        """The projection norms bpr_forward adds to every sample's l2 (model.py:4223-4287 text)."""
        return torch.norm(self.weight_q.weight, p=2) ** 2 + torch.norm(self.weight_k.weight, p=2) ** 2

    def bpr_forward(self, users, pos_items, neg_items):
        users_r, pos_r, neg_r, l2 = NGCF.bpr_forward(self, users, pos_items, neg_items)
        l2 = l2 + torch.norm(self.weight_q.weight, p=2) ** 2 + torch.norm(self.weight_k.weight, p=2) ** 2
        return users_r, pos_r, neg_r, l2


class IMCGAE(BasicModel):
    """model.py:4300-4345: every node's row is [personal | general | identical]
    (3 d wide: its own vector, one vector shared by all users or by all items, one
    shared by everybody); each layer drops nodes at rate dropout - 0.1 i, multiplies
    by the normalised adjacency, and the layers are summed with weights 1 / (i + 2).

    The reference pushes all 3 d columns through gspmm.  Two of the three blocks are
    one vector repeated on every row, and A (s g^T) = (A s) g^T: they stay rank one
    through every layer, so only the personal block takes the d-wide SpMM; the other
    two follow from one scalar per node and layer (a width-1 product with the same
    matrix and the same node masks).  Users and items swap general vectors at every
    layer (the graph is bipartite), which the even / odd sums below account for."""

    def __init__(self, model_config):
        super().__init__(model_config)
        self.embedding_size = model_config['embedding_size']
        self.n_layers = model_config['n_layers']
        self.dropout = model_config['dropout']
        self.embedding = nn.Embedding(self.n_users + self.n_items + 3, self.embedding_size)
        self.norm_adj = self.generate_graph(model_config['dataset'])
        normal_(self.embedding.weight, std=0.1)
        self.to(device=self.device)

    def generate_graph(self, dataset):
        return LightGCN.generate_graph(self, dataset)

    def node_dropout_mask(self, layer):
        """F.dropout of a vector of ones at rate dropout - 0.1 * layer (model.py:4331-4332),
        or None when it is the identity.  config['dropout_rng'] = 'cpu' draws it from the
        CPU generator, as a run of the reference on the CPU does."""
        p = self.dropout - 0.1 * layer
        if not self.training or p <= 0:
            return None
        n = self.n_users + self.n_items
        if self.config.get('dropout_rng', 'device') == 'cpu':
            return F.dropout(torch.ones(n, dtype=torch.float32), p=p, training=True).to(self.device)
        return F.dropout(torch.ones(n, dtype=torch.float32, device=self.device), p=p, training=True)

    def get_rep(self):
        U, n = self.n_users, self.n_users + self.n_items
        # tail rows: the identical vector, the users' general vector, the items' (one split: its
        # backward is one concatenation, not a table-sized zero fill per selected row)
        x, tail = torch.split(self.embedding.weight, [n, 3])
        dev = x.device
        # the repeated blocks' scalar per node (a width-1 product per layer, ops.spmv); no gradient
        s = torch.ones(n, dtype=torch.float32, device=dev)
        acc = x
        even, odd = s, None  # sums of s_l / (l + 1) over even / odd layers l
        for i in range(self.n_layers):
            mask = self.node_dropout_mask(i)
            if mask is not None:
                x = x * mask[:, None]
                s = s * mask
            x = ops.gspmm(self.norm_adj, 'mul', 'sum', x, self.norm_vals)
            with torch.no_grad():
                s = ops.spmv(self.norm_adj, s, self.norm_vals)
            inv = 1. / float(i + 2)
            acc = torch.add(acc, x, alpha=inv)
            if i % 2 == 0:  # layer i + 1 is odd
                odd = s * inv if odd is None else torch.add(odd, s, alpha=inv)
            else:
                even = torch.add(even, s, alpha=inv)
        # a user's general block: its own side's vector on even layers, the items' on odd ones.
        # Per node the coefficients of (identical, users' general, items' general):
        cached = self.__dict__.get('_is_user')
        if cached is None or cached[0] != (U, n, dev):
            cached = self._is_user = ((U, n, dev), (torch.arange(n, device=dev) < U)[:, None])
        is_user = cached[1]
        e = even[:, None]
        o = torch.zeros_like(e) if odd is None else odd[:, None]
        coef = torch.cat([e + o, torch.where(is_user, e, o), torch.where(is_user, o, e)], dim=1)
        general = ops.coef_product(coef[:, 1:], tail[1:])
        identical = ops.coef_product(coef[:, :1], tail[:1])
        return torch.cat([acc, general, identical], dim=1)

    def bpr_forward(self, users, pos_items, neg_items):
        return NGCF.bpr_forward(self, users, pos_items, neg_items)

    def bpr_loss(self, users, pos_items, neg_items, need_l2=True):
        return NGCF.bpr_loss(self, users, pos_items, neg_items, need_l2)

    def predict(self, users, rep=None):
        return LightGCN.predict(self, users, rep)


def graph_rank_nodes(dataset, ranking_metric):
    """utils.py:186-215 for the 'degree' and 'sort'/'greedy' metrics (feature_ratio < 1)."""
    pairs = train_pairs(dataset)
    U, I = dataset.n_users, dataset.n_items
    u, i = pairs[:, 0], pairs[:, 1]
    row = np.concatenate([u, i + U])
    col = np.concatenate([i + U, u])
    rp, ci, v, _ = csr_from_coo(row, col, U + I, U + I, None, dedup=True, want_eid=False)
    deg = row_sums(rp, v).astype(np.float64)
    if ranking_metric == 'degree':
        metrics = deg
    elif ranking_metric in ('sort', 'greedy'):
        # column sums of the l1 row-normalised adjacency (sklearn normalize, utils.py:199-201)
        rows = np.repeat(np.arange(U + I), np.diff(rp))
        metrics = np.bincount(ci, weights=v / deg[rows], minlength=U + I)
    else:
        raise ValueError(f'ranking metric {ranking_metric} not supported')
    return np.argsort(metrics[:U])[::-1].copy(), np.argsort(metrics[U:])[::-1].copy()
