"""igr.dist - edge-range sharded bipartite propagation across the GPUs of a node.

The reference has no parallelism; this is the build's
own multi-GPU layer.  Partition:

  * users are cut into `world` contiguous ranges with balanced edge counts;
    rank k owns user rows U_k, every edge of those users (both directions)
    and X[U_k];
  * the item block X[I] is replicated on every rank.

One propagation layer Y = A X of the symmetric-normalised bipartite graph:

  user rows   Y[U_k] = A[U_k, I] X[I]          local and complete
  item rows   Y^k[I] = A[I, U_k] X[U_k]         partial over U_k
              Y[I]   = sum_k Y^k[I]             RCCL all-reduce (sum) over xGMI

The all-reduce is issued right after the item-side SpMM and overlaps the
user-side SpMM (RCCL runs on its own stream).  The collective moves only
I x d floats per layer (256 MB at I = 1M, d = 64), never the user block.
The smaller side should be the replicated one; `replicate` picks it.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import ops
from .graph import Graph, TiledGraph, csr_from_coo, sym_norm_values

MALL_BYTES = 256 << 20  # MI355X Infinity Cache


def balanced_ranges(degree, world):
    """Contiguous cut of rows into `world` ranges with ~equal edge counts."""
    cum = np.concatenate([[0], np.cumsum(degree, dtype=np.int64)])
    targets = cum[-1] * np.arange(1, world) / world
    cuts = np.clip(np.searchsorted(cum, targets, side='left'), 1, len(cum) - 1)
    # take the row boundary nearest to each target
    cuts = np.where(targets - cum[cuts - 1] < cum[cuts] - targets, cuts - 1, cuts)
    cuts = np.maximum.accumulate(cuts)
    bounds = np.concatenate([[0], cuts, [len(degree)]]).astype(np.int64)
    return [(int(bounds[k]), int(bounds[k + 1])) for k in range(world)]


class BipartiteShard:
    """Rank-local blocks of D^-1/2 A D^-1/2 for a user range [u0, u1).

    pairs: all (user, item) interactions (every rank sees the same list);
    values follow utils.generate_daj_mat + LightGCN.generate_graph exactly
    (duplicates summed, fp32 degrees, numpy float32 pow, (dinv_r*a)*dinv_c).
    """

    def __init__(self, pairs, n_users, n_items, rank, world, device, degree=None, d=64, item_tiles='auto'):
        self.n_users, self.n_items = n_users, n_items
        self.rank, self.world = rank, world
        u, i = pairs[:, 0], pairs[:, 1]
        if degree is None:
            # duplicates count with multiplicity, as scipy sums them into the degree
            degree = np.bincount(u, minlength=n_users).astype(np.float32)
            degree = np.concatenate([degree, np.bincount(i, minlength=n_items).astype(np.float32)])
        self.degree = degree
        self.dinv = np.power(np.maximum(np.float32(1.), degree), np.float32(-0.5)).astype(np.float32)
        self.ranges = balanced_ranges(degree[:n_users], world)
        u0, u1 = self.ranges[rank]
        self.u0, self.u1 = u0, u1
        mine = (u >= u0) & (u < u1)
        lu, li = u[mine] - u0, i[mine]
        nu = u1 - u0
        # user block: rows = local users, cols = items
        rp, ci, v, _ = csr_from_coo(lu, li, nu, n_items, None, dedup=True, want_eid=False)
        dinv_u, dinv_i = self.dinv[u0:u1], self.dinv[n_users:]
        vals = sym_norm_values(rp, ci, v, dinv_u, dinv_i)
        self.user_block = Graph(rp, ci, nu, n_items, device=device)
        self.user_vals = torch.from_numpy(vals).to(device)
        # item block: rows = items, cols = local users
        rp2, ci2, v2, _ = csr_from_coo(li, lu, n_items, nu, None, dedup=True, want_eid=False)
        vals2 = sym_norm_values(rp2, ci2, v2, dinv_i, dinv_u)
        self.item_block = Graph(rp2, ci2, n_items, nu, device=device)
        self.item_vals = torch.from_numpy(vals2).to(device)
        self.local_nnz = self.user_block.nnz + self.item_block.nnz
        # Item rows gather the (large) user table: cut it into source tiles of
        # ~640 MB so each pass gathers from a slice the Infinity Cache can hold,
        # accumulating in place into the (small) item output.  Measured on MI355X
        # at 10M x 1M, d = 64: 8.2 -> 7.7 ms (T = 4); more tiles cost more
        # output passes than they save.
        T = item_tiles
        if T == 'auto':
            table, out = nu * d * 4, n_items * d * 4
            T = int(min(8, -(-table // (640 << 20)))) if table > 4 * max(out, MALL_BYTES) else 1
        self.item_tiles = max(1, int(T))
        self.item_tiled = None
        if self.item_tiles > 1:
            b = [int(round(k * nu / self.item_tiles)) for k in range(self.item_tiles + 1)]
            self.item_tiled = TiledGraph(self.item_block.host(), n_items, nu, b, device)
            self.item_tile_vals = self.item_tiled.tile_values(self.item_vals)

    def launches(self):
        """The SpMM launches of one layer: (name, graph, source, n_rows, nnz)."""
        out = []
        if self.item_tiled is not None:
            for t, g in enumerate(self.item_tiled.tiles):
                out.append((f'item{t}', g, 'users', g.n_rows, g.nnz))
        else:
            out.append(('item', self.item_block, 'users', self.item_block.n_rows, self.item_block.nnz))
        out.append(('user', self.user_block, 'items', self.user_block.n_rows, self.user_block.nnz))
        return out

    def layer(self, x_users, x_items, y_users=None, y_items=None, group=None, spmm=None, hook=None):
        """One layer: returns (Y[U_k], Y[I]) with Y[I] all-reduced across ranks.
        `spmm` defaults to the HIP kernel (the CPU gloo tests pass the oracle);
        `hook(i, 'start'|'end')` brackets each SpMM launch (bench timing)."""
        hook = hook or (lambda i, ph: None)
        if spmm is None and self.item_tiled is not None:
            tg = self.item_tiled
            if y_items is None:
                y_items = torch.empty(self.n_items, x_users.shape[1], dtype=torch.float32, device=x_users.device)
            for t, (g, v) in enumerate(zip(tg.tiles, self.item_tile_vals)):
                hook(t, 'start')
                ops.spmm(g, x_users[tg.bounds[t]:tg.bounds[t + 1]], v, out=y_items,
                         epi=None if t == 0 else ops.epilogue(beta=1.0, add=y_items))
                hook(t, 'end')
            n_item = len(tg.tiles)
        else:
            spmm = ops.spmm if spmm is None else spmm
            hook(0, 'start')
            y_items = spmm(self.item_block, x_users, self.item_vals, out=y_items)
            hook(0, 'end')
            n_item = 1
        work = None
        if self.world > 1:
            work = dist.all_reduce(y_items, op=dist.ReduceOp.SUM, group=group, async_op=True)
        hook(n_item, 'start')
        y_users = (spmm or ops.spmm)(self.user_block, x_items, self.user_vals, out=y_users)
        hook(n_item, 'end')
        if work is not None:
            work.wait()
        return y_users, y_items
