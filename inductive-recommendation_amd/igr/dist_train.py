"""igr.dist_train - IGCN training sharded across the GPUs of a node.

The reference trains on one device (trainer.py:518-561); this is the build's
data-parallel restatement of the same step over the partition of igr.dist:

  * rank k owns the users U_k = [u0, u1) (edge-balanced ranges), their rows of
    the adjacency (both directions) and their user FEATURES; the item
    features and the two general features are replicated;
  * the rank's embedding table is E_k = [E[U_k]; E[items]; E[gen_u]; E[gen_i]]
    (feature_ratio = 1: user u's feature is u, item i's is U + i,
    IGCN.generate_feat / model.py:4139-4175);
  * one feature graph per rank, rows [local users; items] x columns E_k: a
    user row reads its items' features and gen_u; an item row reads its local
    users' features (+ gen_i on rank 0 only), so its output is a partial sum.

Forward (IGCN.get_rep, model.py:4188-4200):
  x0 = F_k E_k                               item rows all-reduced (async,
                                             overlapping layer 1's item side)
  x_{l+1} = A x_l                            BipartiteShard.layer: one item
                                             all-reduce per layer
  rep_k = [mean_l x_l[U_k]; mean_l x_l[I]]   items identical on every rank
Backward (A symmetric, so the same blocks):
  dX_L  = g / (L+1), item part all-reduced once (every rank's batch items)
  dX_l  = A dX_{l+1} + g / (L+1)             each rank folds its own item terms
                                             into its partial before the reduce
  dE_k  = F_k^T dX_0                         owned user-feature rows complete;
                                             replicated rows partial
Step (IGCNTrainer.step, trainer.py:531-561): every rank samples its batch
from its own users (device sampler), loss_k = (bpr + l2_reg l2 + aux_reg aux)
/ world, backward, ONE all-reduce of the replicated rows' gradients and w's
(DDP-style), fused Adam on every rank (identical replicated updates).  The
global step is a batch of world x B samples (weak scaling, as DDP).

The SpMM is pluggable (`spmm=`) so the CPU gloo tests run the same code with
the oracle; on a GPU it is the HIP kernel.
"""
import numpy as np
import torch
import torch.nn as nn

from . import comm, ops
from .dist import BipartiteShard, _hip_spmm
from .graph import Graph, count_ids, csr_from_coo, select_id_range
from .model import train_pairs


def _allreduce(t, group, async_op=False):
    return comm.all_reduce_sum(t, group, async_op=async_op)


class FeatureShard:
    """The rank's rows of IGCN's feature graph over its embedding table E_k.

    Rows [0, n_k) are the local users, rows n_k + i the items; columns index
    E_k: local user features [0, n_k), item features n_k + i, gen_u at
    n_k + I, gen_i at n_k + I + 1.  row_sum is the GLOBAL row sum of the
    reference's feature matrix (duplicates counted, + 1 for the general
    feature), so the values equal the unsharded model's."""

    def __init__(self, pairs, n_users, n_items, u0, u1, rank, device, degree=None):
        """degree: float32 [U + I] interaction counts of the WHOLE graph when the caller has
        them already (BipartiteShard.degree: counted once, by all ranks together); counted here
        otherwise."""
        U, I = n_users, n_items
        nk = u1 - u0
        u, i = pairs[:, 0], pairs[:, 1]
        lu, li = select_id_range(u, i, u0, u1)
        rows = [lu, nk + li, np.arange(nk)]
        cols = [nk + li, lu, np.full(nk, nk + I)]
        if rank == 0:  # the general item feature enters the item rows' sum once
            rows.append(nk + np.arange(I))
            cols.append(np.full(I, nk + I + 1))
        rp, ci, _, _ = csr_from_coo(np.concatenate(rows), np.concatenate(cols), nk + I, nk + I + 2, None,
                                    dedup=True, want_eid=False)
        self.graph = Graph(rp, ci, nk + I, nk + I + 2, device=device)
        if degree is None:
            deg_u, deg_i = count_ids(u, U).astype(np.float32), count_ids(i, I).astype(np.float32)
        else:
            deg_u, deg_i = degree[:U], degree[U:]
        self.row_sum = torch.from_numpy(np.concatenate([deg_u[u0:u1], deg_i]) + np.float32(1.)).to(device)
        self.n_local, self.n_items = nk, I

    def row_values(self, alpha):
        """Per-row value row_sum ** ((alpha - 1)/2 - 0.5) (IGCN.update_feat_mat, model.py:4127-4130)."""
        ex = (alpha - 1.) / 2. - 0.5
        return self.row_sum.double().pow(ex).float() if not self.row_sum.is_cuda else \
            ops.feat_row_values(self.row_sum, ex)

    def edge_values(self, alpha):
        """The same values per edge (CPU / explicit path)."""
        rv = self.row_values(alpha)
        h = self.graph.host()
        rows = torch.from_numpy(np.repeat(np.arange(self.graph.n_rows), np.diff(h['row_ptr']))).to(rv.device)
        return rv[rows].contiguous()


class ShardedPropagate(torch.autograd.Function):
    """rep_k = [rep[U_k]; rep[I]] of IGCN.get_rep on the rank's shard (see module doc).

    The user rows' running layer mean is kept by the SpMM epilogue (the last
    layer divides by L+1); the item rows (I x d, complete only after their
    reduce) are accumulated after it.  aux = (users, pos, neg) (local user
    ids) also returns the aux BPR term on E_k with w, its gradient added into
    dE_k in place (as ops.PropagateRows)."""

    @staticmethod
    def forward(ctx, emb, w, model, fvals, aux):
        sh, fs, L, spmm, group = model.shard, model.feat, model.n_layers, model.spmm, model.group
        ctx.model, ctx.fvals, ctx.aux = model, fvals, aux
        ctx.save_for_backward(emb if aux is not None else None, w)
        nk = fs.n_local
        d = emb.shape[1]
        L1 = float(L + 1)
        x0 = torch.empty(nk + fs.n_items, d, dtype=torch.float32, device=emb.device)
        acc = torch.empty_like(x0)
        model.feat_spmm(fs.graph, emb, fvals, x0, acc=acc)  # acc = x0 (item rows partial until reduced)
        xi = x0[nk:]
        pend = [_allreduce(xi, group, async_op=True)] if model.world > 1 else []
        bufs = [torch.empty_like(x0), torch.empty_like(x0)]
        x = x0
        for layer in range(L):
            y = bufs[layer % 2]
            last = layer == L - 1
            sh.layer(x[:nk], x[nk:], y_users=y[:nk], y_items=y[nk:], group=group, spmm=spmm, pending=pend,
                     acc_users=acc[:nk], acc_div=L1 if last else 1.0)
            if layer == 0:
                acc[nk:].copy_(xi)  # x0's item rows are complete once the first layer has waited
            pend = []
            acc[nk:].add_(y[nk:])
            x = y
        for wk in pend:
            wk.wait()
        if L == 0:
            acc[nk:].copy_(xi)
        else:
            acc[nk:].div_(L1)
        aux_loss = None
        if aux is not None:
            aux_loss = model.aux_forward(emb, w, aux)
        return (acc, aux_loss) if aux is not None else acc

    @staticmethod
    def backward(ctx, g, g_aux=None):
        model, fvals = ctx.model, ctx.fvals
        emb, w = ctx.saved_tensors
        sh, fs, L, spmm, group = model.shard, model.feat, model.n_layers, model.spmm, model.group
        nk = fs.n_local
        L1 = float(L + 1)
        g = g.contiguous()
        gu, gi = g[:nk], g[nk:]
        x = torch.empty_like(g)
        x[nk:].copy_(gi)
        if model.world > 1:
            _allreduce(x[nk:], group)  # every rank's batch items
        torch.div(gu, L1, out=x[:nk])
        x[nk:].div_(L1)
        bufs = [torch.empty_like(g), x]
        for layer in range(L):
            y = bufs[layer % 2]
            sh.layer(x[:nk], x[nk:], y_users=y[:nk], y_items=y[nk:], group=group, spmm=spmm, add_users=gu,
                     add_items=gi, beta=1.0 / L1)
            x = y
        demb = torch.empty(fs.graph.n_cols, g.shape[1], dtype=torch.float32, device=g.device)
        model.feat_spmm(fs.graph.reverse(), x, fvals, demb, reverse=True)
        dw = None
        if ctx.aux is not None and g_aux is not None:
            dw = model.aux_backward(emb, w, ctx.aux, g_aux, demb)
        return demb, dw, None, None, None


def _batch_masks(model, rows_u, items_all):
    """Bitmaps of the rows the batch-row layer reads one layer below (HIP path):
    local users = rows_u + the local neighbours of every rank's batch items;
    items = every rank's batch items + the item neighbours of every rank's batch
    users (OR over ranks: an item's value is the sum of all ranks' partials, so
    every rank must compute its partial wherever any rank reads it)."""
    sh = model.shard
    mu = ops.column_mask(sh.item_block, items_all, extra=rows_u)
    mi = ops.column_mask(sh.user_block, rows_u, extra=items_all)
    if model.world > 1:
        allm = torch.empty(model.world * mi.numel(), dtype=mi.dtype, device=mi.device)
        comm.all_gather_into(allm, mi, model.group)
        allm = allm.view(model.world, -1)
        mi = allm[0].clone()
        for k in range(1, model.world):
            mi.bitwise_or_(allm[k])
    return mu, mi


class ShardedPropagateRows(torch.autograd.Function):
    """rep at the local batch rows [users (local ids); items_b] with the LAST
    layer computed only there (the single-GPU ops.PropagateRows on the shard).

    Forward: x_0 .. x_{L-1} in full (one item all-reduce per layer), then
      users  rep[u] = ((A x)[u] + x[u] + sum_{l<L-1} x_l[u]) / (L+1)   spmm_rows, local
      items  every rank's batch items are all-gathered; each rank computes its
             partial (A x)[i] at all of them on its item block (spmm_rows) and
             ONE small all-reduce (world x 2B x d) completes them.
    Backward, first layer as masked pulls (no full SpMM):
      users  dX[U_k] = A[U_k, I] G_I (every rank's item gradients, all-gathered)
             + G at the local batch users
      items  dX[I]   = sum_k (A[I, U_k] G_{U_k} + own item terms)  (one I x d reduce)
    then L-1 full layers with the batch terms scattered back in, and F^T."""

    @staticmethod
    def forward(ctx, emb, w, model, fvals, aux, rows_u, items_b):
        sh, fs, L, spmm, group = model.shard, model.feat, model.n_layers, model.spmm, model.group
        R = model.rowops
        ctx.model, ctx.fvals, ctx.aux = model, fvals, aux
        nk, I = fs.n_local, fs.n_items
        d = emb.shape[1]
        L1 = float(L + 1)
        world = model.world
        if world > 1:
            items_all = torch.empty(world * items_b.numel(), dtype=torch.int64, device=emb.device)
            comm.all_gather_into(items_all, items_b, group)
        else:
            items_all = items_b
        ctx.save_for_backward(emb if aux is not None else None, w, rows_u, items_b, items_all)
        x = torch.empty(nk + I, d, dtype=torch.float32, device=emb.device)
        model.feat_spmm(fs.graph, emb, fvals, x)
        pend = [_allreduce(x[nk:], group, async_op=True)] if world > 1 else []
        # the layer under the batch-row layer only where that layer reads it (HIP path)
        masks = _batch_masks(model, rows_u, items_all) if (L > 1 and spmm is _hip_spmm) else None
        ctx.masks = masks
        su = si = None
        bufs = [torch.empty_like(x), torch.empty_like(x)]
        for layer in range(L - 1):
            y = bufs[layer % 2]
            lm = ('row',) + masks if (masks is not None and layer == L - 2) else None
            sh.layer(x[:nk], x[nk:], y_users=y[:nk], y_items=y[nk:], group=group, spmm=spmm, pending=pend,
                     masks=lm)
            pend = []
            gu, gi = R.gather(x[:nk], rows_u), R.gather(x[nk:], items_b)
            su = gu if su is None else su.add_(gu)
            si = gi if si is None else si.add_(gi)
            x = y
        for wk in pend:
            wk.wait()
        rep_u = R.rows(sh.user_block, x[nk:], rows_u, sh.user_vals, add_g=x[:nk], add_i=su, scale=1.0 / L1)
        part = R.rows(sh.item_block, x[:nk], items_all, sh.item_vals)
        if world > 1:
            _allreduce(part, group)
        own = part[model.rank * items_b.numel():(model.rank + 1) * items_b.numel()]
        rep_i = own.add_(R.gather(x[nk:], items_b))
        if si is not None:
            rep_i.add_(si)
        rep_i.div_(L1)
        rep = torch.cat([rep_u, rep_i])
        aux_loss = None
        if aux is not None:
            aux_loss = model.aux_forward(emb, w, aux)
        return (rep, aux_loss) if aux is not None else rep

    @staticmethod
    def backward(ctx, g, g_aux=None):
        model, fvals = ctx.model, ctx.fvals
        emb, w, rows_u, items_b, items_all = ctx.saved_tensors
        sh, fs, L, spmm, group = model.shard, model.feat, model.n_layers, model.spmm, model.group
        R = model.rowops
        nk, I = fs.n_local, fs.n_items
        B = rows_u.numel()
        L1 = float(L + 1)
        gs = g.contiguous() / L1
        gu, gi = gs[:B], gs[B:]
        if model.world > 1:
            gi_all = torch.empty(model.world * gi.shape[0], gi.shape[1], dtype=gi.dtype, device=gi.device)
            comm.all_gather_into(gi_all, gi.contiguous(), group)
        else:
            gi_all = gi
        x = torch.empty(nk + I, gs.shape[1], dtype=torch.float32, device=gs.device)
        R.pull(sh.user_block, items_all, gi_all, sh.user_vals, out=x[:nk])
        R.scatter(x[:nk], rows_u, gu)
        R.pull(sh.item_block, rows_u, gu, sh.item_vals, out=x[nk:])
        R.scatter(x[nk:], items_b, gi)
        if model.world > 1:
            _allreduce(x[nk:], group)
        if L > 1:
            gi_dense = torch.zeros(I, gs.shape[1], dtype=torch.float32, device=gs.device)
            R.scatter(gi_dense, items_b, gi)  # own item terms, added to each partial before its reduce
            bufs = [torch.empty_like(x), x]
            for layer in range(L - 1):
                y = bufs[layer % 2]
                # dX_{L-1} is zero off the batch masks: the first reverse layer reads only them
                lm = ('col',) + ctx.masks if (ctx.masks is not None and layer == 0) else None
                sh.layer(x[:nk], x[nk:], y_users=y[:nk], y_items=y[nk:], group=group, spmm=spmm,
                         add_items=gi_dense, beta=1.0, masks=lm)
                R.scatter(y[:nk], rows_u, gu)
                x = y
        demb = torch.empty(fs.graph.n_cols, gs.shape[1], dtype=torch.float32, device=gs.device)
        model.feat_spmm(fs.graph.reverse(), x, fvals, demb, reverse=True)
        dw = None
        if ctx.aux is not None and g_aux is not None:
            dw = model.aux_backward(emb, w, ctx.aux, g_aux, demb)
        return demb, dw, None, None, None, None, None


class _HipRowOps:
    """The row kernels of the batch-row path (the CPU gloo tests pass a numpy restatement)."""

    @staticmethod
    def rows(g, x, rows, vals, add_g=None, add_i=None, scale=1.0):
        return ops.spmm_rows(g, x, rows, vals, add_g=add_g, add_i=add_i, scale=scale)

    @staticmethod
    def pull(g, rows, src, vals, out):
        return ops.spmm_pull(g, rows, src, vals, out=out)

    @staticmethod
    def gather(x, idx):
        return ops.gather_rows(x, idx)

    @staticmethod
    def scatter(dst, idx, src):
        return ops.scatter_add_rows(dst, idx, src)


class ShardedIGCN(nn.Module):
    """IGCN (model.py:4107-4220) on one rank's shard; feature_ratio = 1."""

    def __init__(self, model_config, rank, world, group=None, spmm=None, rowops=None):
        super().__init__()
        ds = model_config['dataset']
        if model_config.get('feature_ratio', 1.) != 1.:
            raise ValueError('ShardedIGCN supports feature_ratio = 1 (every node has its own feature)')
        self.config = model_config
        self.name = 'IGCN'
        self.device = model_config['device']
        self.n_users, self.n_items = ds.n_users, ds.n_items
        self.embedding_size = d = model_config['embedding_size']
        self.n_layers = model_config['n_layers']
        self.dropout = model_config['dropout']
        self.alpha, self.delta = 1., model_config.get('delta', 0.99)
        self.rank, self.world, self.group = rank, world, group
        self.spmm = spmm or _hip_spmm
        self.rowops = rowops or _HipRowOps
        self.hip = spmm is None
        # last layer only at the batch rows (ShardedPropagateRows); 'batch_rep' False = full layers
        self.batch_rows = bool(model_config.get('batch_rep', True)) and self.n_layers > 0
        pairs = train_pairs(ds)
        # set-up divided among the ranks: each counts one slice of the pairs, one host all-reduce
        # of the degrees, then every rank sorts only its own users' interactions
        self.shard = BipartiteShard.from_stream(pairs[:, 0], pairs[:, 1], self.n_users, self.n_items, rank, world,
                                                self.device, group=group, d=d)
        self.u0, self.u1 = self.shard.u0, self.shard.u1
        self.feat = FeatureShard(pairs, self.n_users, self.n_items, self.u0, self.u1, rank, self.device,
                                 degree=self.shard.degree)
        self.n_local = self.u1 - self.u0
        self.embedding = nn.Embedding(self.feat.graph.n_cols, d)
        nn.init.normal_(self.embedding.weight, std=0.1)  # model.py:4124
        self.w = nn.Parameter(torch.ones([d], dtype=torch.float32, device=self.device))
        self.to(device=self.device)
        self.update_feat_mat()
        self._drop_step = -1
        self._drop_seed = int(model_config.get('seed', 0)) & (2 ** 63 - 1)

    # ---------------------------------------------------------------- parameters
    def load_full_embedding(self, full):
        """Take this rank's rows of an unsharded (U + I + 2) x d table (same layout as IGCN's)."""
        U = self.n_users
        with torch.no_grad():
            self.embedding.weight.copy_(torch.cat([full[self.u0:self.u1], full[U:]]).to(self.device))

    def replicated_rows(self):
        return slice(self.n_local, self.feat.graph.n_cols)

    def update_feat_mat(self):
        self.feat_base = self.feat.row_values(self.alpha)
        self._edge_vals = None

    def feat_mat_anneal(self):
        self.alpha *= self.delta
        self.update_feat_mat()

    def feat_values(self):
        """ScaledWeights on the GPU (dropout drawn in the SpMM with a rank-distinct
        key: every rank's edges are distinct edges); explicit values otherwise."""
        if not self.hip:
            if self.training and self.dropout > 0:
                raise NotImplementedError('the CPU restatement path runs without dropout')
            if self._edge_vals is None:
                self._edge_vals = self.feat.edge_values(self.alpha)
            return self._edge_vals
        if self.training and self.dropout > 0:
            self._drop_step += 1
            seed = (self._drop_seed * 0x9E3779B97F4A7C15 + self.rank + 1) & (2 ** 63 - 1)
            return ops.ScaledWeights(self.feat_base, None, 1.0 - self.dropout, seed, self._drop_step)
        return ops.ScaledWeights(self.feat_base)

    def feat_spmm(self, g, x, fvals, out, reverse=False, acc=None):
        """out = F_w x (reverse: F_w^T x); acc = out via the epilogue when given."""
        if isinstance(fvals, ops.ScaledWeights):
            epi = None if acc is None else ops.epilogue(acc=acc, acc_mode=1)
            return ops.spmm_scaled(g, x, fvals.transposed() if reverse else fvals, out=out, epi=epi)
        if acc is None:
            return self.spmm(g, x, fvals, out, False)
        return self.spmm(g, x, fvals, out, False, acc=acc, acc_mode=1)

    # ---------------------------------------------------------------- model surface
    def get_rep(self):
        """[rep[U_k]; rep[I]] (rows of IGCN.get_rep owned / replicated here)."""
        return ShardedPropagate.apply(self.embedding.weight, self.w, self, self.feat_values(), None)

    def bpr_aux_loss(self, users, pos_items, neg_items, a_users, a_pos, a_neg):
        """IGCNTrainer terms on the local batch (users are LOCAL ids); the aux
        term's gradient joins dE_k inside the propagation backward."""
        aux_idx = tuple(t.to(torch.int64).contiguous() for t in (a_users, a_pos, a_neg))
        if self.batch_rows:
            users, pos_items, neg_items = (t.to(torch.int64).contiguous() for t in (users, pos_items, neg_items))
            items_b = torch.cat([pos_items, neg_items])
            rep, aux = ShardedPropagateRows.apply(self.embedding.weight, self.w, self, self.feat_values(), aux_idx,
                                                  users, items_b)
            iu, ip, ineg = ops.batch_positions(users.numel(), users.device)
            bpr, l2 = ops.bpr_loss(rep, iu, ip, ineg, 0, 0, distinct=True)
            return bpr, l2, aux
        rep, aux = ShardedPropagate.apply(self.embedding.weight, self.w, self, self.feat_values(), aux_idx)
        bpr, l2 = ops.bpr_loss(rep, users, pos_items, neg_items, 0, self.n_local)
        return bpr, l2, aux

    def aux_forward(self, emb, w, aux):
        """Mean aux BPR loss on E_k with w (trainer.py:542-549); item features at n_local."""
        au, ap, an = aux
        loss = torch.empty(au.numel(), dtype=torch.float32, device=emb.device)
        ops._bpr_call(au.numel(), emb.shape[1], au, ap, an, 0, self.n_local, emb, w, loss, None, 0.0, 0.0, None, None,
                      None, 0, None, None)
        return loss.mean()

    def aux_backward(self, emb, w, aux, g_aux, demb):
        """Adds the aux term's gradient into demb in place; returns d w."""
        au, ap, an = aux
        dw = torch.zeros_like(w)
        g_aux = g_aux.float().contiguous()
        ops._bpr_call(au.numel(), emb.shape[1], au, ap, an, 0, self.n_local, emb, w, None, None, 1.0 / au.numel(), 0.0,
                      g_aux, None, demb, demb.stride(0), dw, ops.rowsort(au, 0, ap, self.n_local, an, self.n_local))
        return dw

    def batch_rep(self, users, items_b):
        """[rep[users]; rep[items_b]] through the batch-row path (no aux term)."""
        return ShardedPropagateRows.apply(self.embedding.weight, self.w, self, self.feat_values(), None,
                                          users.to(torch.int64).contiguous(), items_b.to(torch.int64).contiguous())

    def sync_grads(self):
        """One all-reduce of the replicated parameters' gradients (item / general rows and w)."""
        if self.world == 1:
            return
        if self.w.grad is None:
            self.w.grad = torch.zeros_like(self.w)
        ge = self.embedding.weight.grad[self.replicated_rows()]
        buf = torch.cat([ge.reshape(-1), self.w.grad.reshape(-1)])
        _allreduce(buf, self.group)
        ge.copy_(buf[:ge.numel()].view_as(ge))
        self.w.grad.copy_(buf[ge.numel():])


class _LocalPairs:
    """The rank's users' training pairs with local user ids (for the device sampler)."""

    def __init__(self, pairs, u0, u1, n_items):
        mine = (pairs[:, 0] >= u0) & (pairs[:, 0] < u1)
        p = pairs[mine].copy()
        p[:, 0] -= u0
        self.train_pairs, self.n_users, self.n_items = p, u1 - u0, n_items

    def __len__(self):
        return len(self.train_pairs)


class ShardedIGCNTrainer:
    """IGCNTrainer.step (trainer.py:531-561) on every rank of a sharded model."""

    def __init__(self, trainer_config, model):
        from .optim import Adam
        from .sampler import DeviceBPRSampler
        self.model = model
        self.config = trainer_config
        self.batch_size = trainer_config['batch_size']
        self.l2_reg, self.aux_reg = trainer_config['l2_reg'], trainer_config['aux_reg']
        seed = int(trainer_config.get('seed', 0))
        local = _LocalPairs(train_pairs(model.config['dataset']), model.u0, model.u1, model.n_items)
        # aux pairs = the dataset itself at feature_ratio = 1 (AuxiliaryDataset), local user ids
        self.sampler = DeviceBPRSampler(local, self.batch_size, model.device, seed=seed * 1000003 + model.rank)
        self.aux_sampler = DeviceBPRSampler(local, self.batch_size, model.device,
                                            seed=(seed + 1) * 1000003 + model.rank)
        self.opt = Adam(model.parameters(), lr=trainer_config['lr'])

    def step(self, users=None, pos=None, neg=None, a_users=None, a_pos=None, a_neg=None):
        m = self.model
        if users is None:
            users, pos, neg = self.sampler.sample(self.batch_size)
            a_users, a_pos, a_neg = self.aux_sampler.sample(self.batch_size)
        bpr, l2, aux = m.bpr_aux_loss(users, pos, neg, a_users, a_pos, a_neg)
        loss = bpr + self.l2_reg * l2 + self.aux_reg * aux
        self.opt.zero_grad()
        (loss / m.world).backward()
        m.sync_grads()
        self.opt.step()
        return loss
