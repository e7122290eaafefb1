"""igr.dist - edge-range sharded bipartite propagation across the GPUs of a node.

The reference has no parallelism; this is the build's own multi-GPU layer.
Partition:

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
The smaller side should be the replicated one: the layer is symmetric in the
two sides, so a caller whose items outnumber its users passes the pairs with
their columns swapped (then 'users' below means the sharded side) -
`sharded_side` / bench.py --replicate.
"""
import os

import numpy as np
import torch
from . import comm, ops
from .graph import Graph, count_ids, csr_from_coo, csr_transpose, select_id_range, sym_norm_values

MALL_BYTES = 256 << 20  # MI355X Infinity Cache


def sharded_side(n_users, n_items, replicate='auto'):
    """'users' or 'items': the side a BipartiteShard cuts into ranges (the other is
    replicated); 'auto' replicates the smaller side."""
    if replicate == 'auto':
        return 'users' if n_users >= n_items else 'items'
    if replicate not in ('items', 'users'):
        raise ValueError(f"replicate must be 'auto', 'items' or 'users', got {replicate!r}")
    return 'users' if replicate == 'items' else 'items'


def _align32(ranges, n):
    """Move the inner boundaries of contiguous ranges to multiples of 32, so a row
    bitmap over the whole range can be handed to each piece as a word offset."""
    b = [0] + [min(n, 32 * int(round(e / 32))) for _, e in ranges[:-1]] + [n]
    b = list(np.maximum.accumulate(b))
    return [(int(b[k]), int(b[k + 1])) for k in range(len(ranges))]


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

    The item block is cut two ways:
      * row chunks (world > 1): each chunk's partial is all-reduced as soon as
        its SpMM is done, so the exchange overlaps the remaining item chunks
        and the user-side SpMM; only the last chunk's reduce is exposed;
      * source tiles (large user tables): each pass gathers from a slice of
        X[U_k] the Infinity Cache can hold, accumulating in place.
    """

    def __init__(self, pairs, n_users, n_items, rank, world, device, degree=None, d=64, item_tiles='auto',
                 item_chunks='auto', local_pairs=None):
        """pairs: int64 [n, 2] or a (users, items) tuple of int64 arrays.  local_pairs
        (with `degree`): (users - u0, items) of this rank's own range only, already
        selected - what from_stream hands over; `pairs` is then not read."""
        self.n_users, self.n_items = n_users, n_items
        self.rank, self.world = rank, world
        # the layer all-reduces its item partials; a test may switch it on at world 1 to run
        # the exchange pattern through a one-rank process group
        self.exchange = world > 1
        if local_pairs is None:
            u, i = (pairs[:, 0], pairs[:, 1]) if isinstance(pairs, np.ndarray) else pairs
        elif degree is None:
            raise ValueError('local_pairs needs the degrees of the whole graph (degree=): a range of the pairs cannot give them')
        if degree is None:
            # duplicates count with multiplicity, as scipy sums them into the degree
            degree = np.concatenate([count_ids(u, n_users), count_ids(i, n_items)]).astype(np.float32)
        self.degree = degree
        self.dinv = np.power(np.maximum(np.float32(1.), degree), np.float32(-0.5)).astype(np.float32)
        self.ranges = balanced_ranges(degree[:n_users], world)
        u0, u1 = self.ranges[rank]
        self.u0, self.u1 = u0, u1
        lu, li = select_id_range(u, i, u0, u1) if local_pairs is None else local_pairs
        nu = u1 - u0
        # user block: rows = local users, cols = items
        rp, ci, v, _ = csr_from_coo(lu, li, nu, n_items, None, dedup=True, want_eid=False)
        dinv_u, dinv_i = self.dinv[u0:u1], self.dinv[n_users:]
        vals = sym_norm_values(rp, ci, v, dinv_u, dinv_i)
        self.user_block = Graph(rp, ci, nu, n_items, device=device)
        self.user_vals = torch.from_numpy(vals).to(device)
        self._user_counts, self._dinv_u, self._dinv_i = v, dinv_u, dinv_i
        self._item_host = None
        # source tiles: ~640 MB slices when the user table dwarfs the item output and the
        # Infinity Cache (measured on MI355X at 10M x 1M, d = 64: 8.2 -> 7.7 ms at T = 4)
        T = item_tiles
        if T == 'auto':
            table, out = nu * d * 4, n_items * d * 4
            T = int(min(8, -(-table // (640 << 20)))) if table > 4 * max(out, MALL_BYTES) else 1
        self.item_tiles = max(1, int(T))
        C = item_chunks
        if C == 'auto':
            C = 4 if world > 1 else 1
        self.item_chunks = max(1, int(C))
        # row chunks with ~equal nnz, cut on the GLOBAL item degrees so every rank
        # all-reduces the same row ranges
        cuts = _align32(balanced_ranges(degree[n_users:], self.item_chunks), n_items)
        col_bounds = [min(nu, 32 * int(round(k * nu / self.item_tiles / 32))) for k in range(self.item_tiles)] + [nu]
        # item block: rows = items, cols = local users.  Each source tile is the transpose
        # of a range of user rows (the user block is sorted, so the transposed rows come
        # out sorted by user); a row chunk is a row range of every tile.
        tile_csr = []
        for t in range(self.item_tiles):
            b0, b1 = col_bounds[t], col_bounds[t + 1]
            tile_csr.append(self._transpose_users(b0, b1))
        self.item_nnz = sum(int(t_rp[-1]) for t_rp, _, _ in tile_csr)
        if self.item_tiles == 1:
            self._item_host = dict(zip(('row_ptr', 'col_idx', 'vals'), tile_csr[0]))
        self.local_nnz = self.user_block.nnz + self.item_nnz
        self.chunks = []  # (r0, r1, [(graph, vals, c0, c1), ...])
        for r0, r1 in cuts:
            tiles = []
            for t, (t_rp, t_ci, t_v) in enumerate(tile_csr):
                e0, e1 = int(t_rp[r0]), int(t_rp[r1])
                g = Graph(t_rp[r0:r1 + 1] - e0, t_ci[e0:e1], r1 - r0, col_bounds[t + 1] - col_bounds[t], device=device)
                tiles.append((g, torch.from_numpy(t_v[e0:e1]).to(device), col_bounds[t], col_bounds[t + 1]))
            self.chunks.append((r0, r1, tiles))

    def _transpose_users(self, b0, b1):
        """(row_ptr, col_idx, vals) of A[I, b0:b1): the item rows over the local users
        [b0, b1), columns relative to b0, values (dinv_i * a) * dinv_u (model.py:91-96)."""
        h = self.user_block.host()
        rp, ci = h['row_ptr'], h['col_idx']
        e0, e1 = int(rp[b0]), int(rp[b1])
        t_rp, t_ci, t_pos = csr_transpose(rp[b0:b1 + 1] - e0, ci[e0:e1], b1 - b0, self.n_items)
        # multi-threaded gather of the duplicate counts into transposed order
        a = torch.from_numpy(self._user_counts[e0:e1]).index_select(0, torch.from_numpy(t_pos)).numpy()
        return t_rp, t_ci, sym_norm_values(t_rp, t_ci, a, self._dinv_i, self._dinv_u[b0:b1])

    @property
    def item_host(self):
        """The whole item block as one host CSR: dict(row_ptr, col_idx, vals)."""
        if self._item_host is None:
            self._item_host = dict(zip(('row_ptr', 'col_idx', 'vals'), self._transpose_users(0, self.u1 - self.u0)))
        return self._item_host

    @classmethod
    def from_stream(cls, users, items, n_users, n_items, rank, world, device, group=None, timings=None,
                    reduce=None, **kw):
        """A shard built from an interaction stream every rank holds (drawn from one
        seed, or read from one file) with the counting and the CSR builds divided
        among the ranks: rank k counts the degrees of the k-th slice of the stream,
        the counts are added up across the ranks (one host all-reduce of
        n_users + n_items integers), and each rank then selects and sorts only the
        interactions of its own user range.  Needs an initialised process group
        when world > 1, unless `reduce` (counts of this rank's slice -> counts of the
        whole stream) is given in place of the all-reduce.  timings: dict that
        receives the seconds of each stage."""
        import time
        t0 = time.perf_counter()
        E = len(users)
        e0, e1 = E * rank // world, E * (rank + 1) // world
        counts = np.concatenate([count_ids(users[e0:e1], n_users), count_ids(items[e0:e1], n_items)])
        if reduce is not None:
            counts = reduce(counts)
        elif world > 1:
            counts = comm.all_reduce_sum_host(counts, group, device)
        degree = counts.astype(np.float32)
        t1 = time.perf_counter()
        u0, u1 = balanced_ranges(degree[:n_users], world)[rank]
        local = select_id_range(users, items, u0, u1)
        t2 = time.perf_counter()
        sh = cls(None, n_users, n_items, rank, world, device, degree=degree, local_pairs=local, **kw)
        if timings is not None:
            timings.update(count_s=t1 - t0, select_s=t2 - t1, build_s=time.perf_counter() - t2)
        return sh

    @property
    def item_block(self):
        """The whole item block as one Graph (built on first use; the layer uses the chunks)."""
        if getattr(self, '_item_block', None) is None:
            h = self.item_host
            self._item_block = Graph(h['row_ptr'], h['col_idx'], self.n_items, self.u1 - self.u0,
                                     device=self.user_block.device)
        return self._item_block

    @property
    def item_vals(self):
        """Values of the whole item block (CSR order), on the device."""
        if getattr(self, '_item_vals', None) is None:
            self._item_vals = torch.from_numpy(self.item_host['vals']).to(self.user_block.device)
        return self._item_vals

    def launches(self):
        """The SpMM launches of one layer: (name, graph, source, n_rows, nnz)."""
        out = []
        for k, (r0, r1, tiles) in enumerate(self.chunks):
            for t, (g, _, _, _) in enumerate(tiles):
                out.append((f'item{k}.{t}', g, 'users', g.n_rows, g.nnz))
        out.append(('user', self.user_block, 'items', self.user_block.n_rows, self.user_block.nnz))
        return out

    def layer(self, x_users, x_items, y_users=None, y_items=None, group=None, spmm=None, hook=None,
              add_users=None, add_items=None, beta=0.0, pending=(), acc_users=None, acc_div=1.0, masks=None,
              defer=False):
        """One layer: returns (Y[U_k], Y[I]) with Y[I] all-reduced across ranks.

        With add_users / add_items: Y[U_k] += beta * add_users and every rank
        adds beta * add_items (its own item terms) to its partial before the
        reduce - the training backward's "+ g/(L+1)" (dist_train.py).
        `pending`: collectives producing x_items, waited for just before the
        user-side SpMM (the item side needs only x_users).  acc_users: the
        user-side epilogue also does acc_users = (acc_users + Y[U_k]) / acc_div
        (the forward's running layer mean).
        masks = (mode, user_bits, item_bits), bitmaps over local users / items:
        mode 'row' computes only the marked output rows (the others are left
        as they were), mode 'col' reads only the marked source rows (the others
        must hold zeros) - dist_train's batch-row step.
        `spmm(g, x, vals, out, accumulate, add=None, beta=0., row_mask=None,
        col_mask=None)` defaults to the HIP kernel (the CPU gloo tests pass the
        oracle); `hook(i, 'start'|'end')` brackets each SpMM launch (bench timing).
        defer: do not wait for this layer's item all-reduces; returns
        (Y[U_k], Y[I], works) instead, and the caller passes `works` as the next
        layer's `pending` - chained layers (x_{l+1} = y_l) then overlap the
        reduce of layer l with the item-side SpMM of layer l+1 as well as with
        the user side of layer l (Y[I] is complete only after the wait, and the
        next layer must write its items into another buffer)."""
        hook = hook or (lambda i, ph: None)
        spmm = spmm or _hip_spmm
        if y_items is None:
            y_items = torch.empty(self.n_items, x_users.shape[1], dtype=torch.float32, device=x_users.device)
        mode, mu, mi = masks if masks is not None else (None, None, None)

        def mk(bits, first):  # the bitmap seen from index `first` on (a multiple of 32)
            return None if bits is None else bits[first // 32:]
        works, i = [], 0
        for r0, r1, tiles in self.chunks:
            yk = y_items[r0:r1]
            for t, (g, v, c0, c1) in enumerate(tiles):
                hook(i, 'start')
                kw = {}
                if mode == 'row':
                    kw['row_mask'] = mk(mi, r0)
                elif mode == 'col':
                    kw['col_mask'] = mk(mu, c0)
                d = x_users.shape[1]
                W = _col_width(d, (c1 - c0) * d * 4) if ITEM_SIDE_COL_SPLIT else d
                for c in range(0, d, W):
                    sl = slice(c, c + W)
                    if t == 0 and add_items is not None:
                        spmm(g, x_users[c0:c1, sl], v, yk[:, sl], False, add=add_items[r0:r1, sl], beta=beta, **kw)
                    else:
                        spmm(g, x_users[c0:c1, sl], v, yk[:, sl], t > 0, **kw)
                hook(i, 'end')
                i += 1
            if self.exchange:
                works.append(comm.all_reduce_sum(yk, group, async_op=True))
        if y_users is None:
            y_users = torch.empty(self.u1 - self.u0, x_items.shape[1], dtype=torch.float32, device=x_items.device)
        for w in pending:
            w.wait()
        hook(i, 'start')
        # wide rows whose item table outgrows the Infinity Cache (d = 256 at 1M
        # items): two passes over 128-column halves, each gathering from a
        # cache-sized slice (same sums, column by column)
        d = x_items.shape[1]
        W = _col_width(d, x_items.shape[0] * d * 4)
        for c in range(0, d, W):
            sl = slice(c, c + W)
            kw = {} if acc_users is None else dict(acc=acc_users[:, sl], acc_mode=2, acc_div=acc_div)
            if mode == 'row':
                kw['row_mask'] = mu
            elif mode == 'col':
                kw['col_mask'] = mi
            if add_users is not None:
                spmm(self.user_block, x_items[:, sl], self.user_vals, y_users[:, sl], False,
                     add=add_users[:, sl], beta=beta, **kw)
            else:
                spmm(self.user_block, x_items[:, sl], self.user_vals, y_users[:, sl], False, **kw)
        hook(i, 'end')
        if defer:
            return y_users, y_items, works
        for w in works:
            w.wait()
        return y_users, y_items

    def propagate(self, x_users, x_items, n_layers, group=None, spmm=None):
        """n_layers chained layers (x_{l+1} = A x_l, LightGCN's get_rep without
        the mean) with each layer's item reduce deferred into the next layer;
        returns the last (Y[U_k], Y[I]), fully reduced."""
        d = x_users.shape[1]
        bu = [torch.empty(self.u1 - self.u0, d, dtype=torch.float32, device=x_users.device) for _ in range(2)]
        bi = [torch.empty(self.n_items, d, dtype=torch.float32, device=x_users.device) for _ in range(2)]
        xu, xi, pend = x_users, x_items, []
        for layer in range(n_layers):
            xu, xi, pend = self.layer(xu, xi, bu[layer % 2], bi[layer % 2], group=group, spmm=spmm,
                                      pending=pend, defer=True)
        for w in pend:
            w.wait()
        return xu, xi


ITEM_SIDE_COL_SPLIT = os.environ.get('IGR_ITEM_COL_SPLIT', '1') == '1'


def _col_width(d, table_bytes):
    """Column width per pass of a wide-row SpMM: 128 when d = 256 and the gathered
    table outgrows the Infinity Cache, so each pass gathers from a slice half as
    large (same sums, column by column); d otherwise."""
    forced = int(os.environ.get('IGR_COL_WIDTH', '0'))  # tuning override (scripts / bench experiments)
    if forced > 0 and d % forced == 0:
        return forced
    return 128 if (d == 256 and table_bytes > MALL_BYTES) else d


def _hip_spmm(g, x, vals, out, accumulate, add=None, beta=0.0, acc=None, acc_mode=0, acc_div=1.0, row_mask=None,
              col_mask=None):
    """out = A x (+ out if accumulate) (+ beta * add), and acc = out (mode 1) or
    acc = (acc + out) / acc_div (mode 2), all in the SpMM epilogue; row_mask /
    col_mask restrict the rows computed / the source rows read."""
    if accumulate:
        add, beta = out, 1.0
    if add is None and acc is None and row_mask is None and col_mask is None:
        return ops.spmm(g, x, vals, out=out)
    return ops.spmm(g, x, vals, out=out, epi=ops.epilogue(beta=beta, add=add, acc=acc, acc_mode=acc_mode,
                                                          acc_div=acc_div, row_mask=row_mask, col_mask=col_mask))
