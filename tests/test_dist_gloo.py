"""Sharded bipartite propagation (igr/dist.py) on CPU with gloo, world sizes 2, 4 and 8.

The partition and the all-reduce exchange are the code under test; the
rank-local SpMM is the oracle (these CPU tests have no HIP device), and the
result is compared with the unsharded oracle propagation."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from igr.dist import BipartiteShard, balanced_ranges
from oracle import igr_oracle as O


def oracle_spmm(g, x, vals, out, accumulate, add=None, beta=0.0, acc=None, acc_mode=0, acc_div=1.0, row_mask=None,
                col_mask=None):
    """The rank-local SpMM restated on the CPU: out = A x (+ out) (+ beta add),
    acc = out (mode 1) / (acc + out) / acc_div (mode 2).  vals are by edge id
    (a reverse graph carries the forward edge ids).  row_mask / col_mask are
    ignored: every row computed and every source read is a superset (unmarked
    rows are never read, unmarked sources hold zeros)."""
    h = g.host()
    v = vals.numpy() if h['edge_id'] is None else vals.numpy()[h['edge_id']]
    A = O.CSR(g.n_rows, g.n_cols, h['row_ptr'], h['col_idx'].astype(np.int64), v)
    y = torch.from_numpy(O.spmm(A, np.ascontiguousarray(x.numpy())))
    if accumulate:
        out.add_(y)
    else:
        out.copy_(y)
    if add is not None:
        out.add_(beta * add)
    if acc is not None:
        if acc_mode == 1:
            acc.copy_(out)
        else:
            acc.add_(out).div_(acc_div)
    return out


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, pairs, U, I, d, q, tiles=1, chunks='auto', layers=1):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        sh = BipartiteShard(pairs, U, I, rank, world, 'cpu', item_tiles=tiles, item_chunks=chunks)
        assert len(sh.chunks) == (4 if chunks == 'auto' else chunks)
        g = torch.Generator().manual_seed(0)
        xu_all = torch.randn(U, d, generator=g)
        xi = torch.randn(I, d, generator=g)
        if layers == 1:
            yu, yi = sh.layer(xu_all[sh.u0:sh.u1].contiguous(), xi, spmm=oracle_spmm)
        else:  # chained layers, each item reduce deferred into the next layer
            yu, yi = sh.propagate(xu_all[sh.u0:sh.u1].contiguous(), xi, layers, spmm=oracle_spmm)
        q.put((rank, sh.u0, sh.u1, yu.numpy(), yi.numpy(), sh.local_nnz))
    except Exception:
        import traceback
        q.put((rank, 'error', traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def test_balanced_ranges():
    deg = np.array([5, 1, 1, 1, 10, 2, 2, 2, 0, 6])
    r = balanced_ranges(deg, 3)
    assert r[0][0] == 0 and r[-1][1] == len(deg)
    assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
    loads = [deg[a:b].sum() for a, b in r]
    assert max(loads) - min(loads) <= deg.max()


@pytest.mark.parametrize('world,tiles,chunks', [(2, 1, 'auto'), (2, 3, 2), (4, 1, 'auto'), (8, 2, 4)])
def test_sharded_layer_matches_unsharded(world, tiles, chunks):
    U, I, E, d = 400, 150, 5000, 16
    rng = np.random.default_rng(0)
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pairs, U, I, d, q, tiles, chunks))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    errs = [r[2] for r in res if r[1] == 'error']
    assert not errs, errs[0]
    res = sorted(res, key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # unsharded reference: full D^-1/2 A D^-1/2 over [users; items]
    A = O.norm_adj(U, I, pairs)
    g = torch.Generator().manual_seed(0)
    x = torch.cat([torch.randn(U, d, generator=g), torch.randn(I, d, generator=g)]).numpy()
    y64 = O.spmm64(A, x)
    assert sum(r[5] for r in res) == A.nnz
    for rank, u0, u1, yu, yi, _ in res:
        np.testing.assert_allclose(yu, y64[u0:u1], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(yi, y64[U:], rtol=1e-5, atol=1e-6)  # every rank holds the reduced items
    assert res[0][1] == 0 and res[-1][2] == U


@pytest.mark.parametrize('world', [2, 4])
def test_chained_layers_with_deferred_reduces(world):
    """BipartiteShard.propagate: three chained layers, each layer's item all-reduce
    waited only by the next layer's user side == (D^-1/2 A D^-1/2)^3 x unsharded."""
    U, I, E, d, L = 300, 120, 4000, 8, 3
    rng = np.random.default_rng(5)
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pairs, U, I, d, q, 2, 2, L)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    errs = [r[2] for r in res if r[1] == 'error']
    assert not errs, errs[0]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = O.norm_adj(U, I, pairs)
    g = torch.Generator().manual_seed(0)
    y = torch.cat([torch.randn(U, d, generator=g), torch.randn(I, d, generator=g)]).numpy().astype(np.float64)
    for _ in range(L):
        y = O.spmm64(A, y)
    for rank, u0, u1, yu, yi, _ in res:
        np.testing.assert_allclose(yu, y[u0:u1], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(yi, y[U:], rtol=1e-5, atol=1e-6)


def test_item_chunks_identical_across_ranks():
    """Every rank must all-reduce the same item row ranges (cut on global degrees)."""
    U, I, E = 1000, 300, 8000
    rng = np.random.default_rng(1)
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)
    cuts = [[(r0, r1) for r0, r1, _ in BipartiteShard(pairs, U, I, r, 4, 'cpu').chunks] for r in range(4)]
    assert all(c == cuts[0] for c in cuts) and len(cuts[0]) == 4
    assert cuts[0][0][0] == 0 and cuts[0][-1][1] == I


# ------------------------------------------------------------------ sharded IGCN training (dist_train.py)

class _DS:
    def __init__(self, pairs, U, I):
        self.train_pairs, self.n_users, self.n_items = pairs, U, I
        self.name = 'synthetic'

    def __len__(self):
        return len(self.train_pairs)


def _igcn_worker(rank, world, port, pairs, U, I, d, L, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from igr.dist_train import ShardedIGCN
        m = ShardedIGCN({'dataset': _DS(pairs, U, I), 'embedding_size': d, 'n_layers': L, 'dropout': 0.3,
                         'device': 'cpu', 'feature_ratio': 1.}, rank, world, spmm=oracle_spmm)
        m.eval()  # no dropout on the CPU restatement path
        g = torch.Generator().manual_seed(0)
        emb = torch.randn(U + I + 2, d, generator=g) * 0.1
        R = torch.randn(U + I, d, generator=g)
        m.load_full_embedding(emb)
        rep = m.get_rep()
        G = torch.cat([R[m.u0:m.u1], R[U:] * (rank + 1)])  # rank-specific item terms: they must be summed
        (rep * G).sum().backward()
        m.sync_grads()
        q.put((rank, m.u0, m.u1, rep.detach().numpy(), m.embedding.weight.grad.numpy()))
    except Exception:
        import traceback
        q.put((rank, 'error', traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,L', [(2, 0), (2, 2), (4, 2), (8, 3)])
def test_sharded_igcn_rep_and_grad_match_unsharded(world, L):
    """World 2, 4 and 8: the sharded forward (feature layer + L layers, item
    all-reduces) and backward (item terms of every rank folded into the reduces,
    replicated gradients all-reduced) equal the unsharded IGCN restatement."""
    rng = np.random.default_rng(4)
    U, I, d = 90, 50, 8
    pairs = np.stack([rng.integers(0, U, 900), rng.integers(0, I, 900)], 1)
    pairs = np.concatenate([pairs, pairs[:20]])  # duplicates
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_igcn_worker, args=(r, world, port, pairs, U, I, d, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != 'error', r[2]
    A = O.norm_adj(U, I, pairs)
    F = O.generate_feat(U, I, pairs)
    fv = O.feat_values(F, 1.0)
    g = torch.Generator().manual_seed(0)
    emb = (torch.randn(U + I + 2, d, generator=g) * 0.1).numpy()
    R = torch.randn(U + I, d, generator=g).numpy()
    rep = O.igcn_rep(A, F, fv, emb, L)
    Gt = np.concatenate([R[:U], R[U:] * sum(k + 1 for k in range(world))])
    grad = O.igcn_grad(A, F, fv, L, Gt)
    tol = dict(rtol=1e-5, atol=1e-6)
    # the item gradients are sums over `world` partials: absolute slack on the scale of the gradient
    gtol = dict(rtol=1e-5, atol=1e-6 * max(1.0, float(np.abs(grad).max())))
    for rank, u0, u1, rep_k, grad_k in res:
        nk = u1 - u0
        np.testing.assert_allclose(rep_k[:nk], rep[u0:u1], **tol)
        np.testing.assert_allclose(rep_k[nk:], rep[U:], **tol)
        np.testing.assert_allclose(grad_k[:nk], grad[u0:u1], **gtol)
        np.testing.assert_allclose(grad_k[nk:], grad[U:], **gtol)


class NumpyRowOps:
    """The batch-row kernels restated with the oracle SpMM (rows / pull) and torch indexing."""

    @staticmethod
    def rows(g, x, rows, vals, add_g=None, add_i=None, scale=1.0):
        y = oracle_spmm(g, x, vals, torch.empty(g.n_rows, x.shape[1]), False)[rows]
        if add_g is not None:
            y = y + add_g[rows]
        if add_i is not None:
            y = y + add_i
        return (y * scale).contiguous()

    @staticmethod
    def pull(g, rows, src, vals, out):
        S = torch.zeros(g.n_cols, src.shape[1]).index_add_(0, rows, src)
        return oracle_spmm(g, S, vals, out, False)

    @staticmethod
    def gather(x, idx):
        return x[idx].contiguous()

    @staticmethod
    def scatter(dst, idx, src):
        return dst.index_add_(0, idx, src)


def _rows_worker(rank, world, port, pairs, U, I, d, L, B, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from igr.dist_train import ShardedIGCN
        m = ShardedIGCN({'dataset': _DS(pairs, U, I), 'embedding_size': d, 'n_layers': L, 'dropout': 0.3,
                         'device': 'cpu', 'feature_ratio': 1.}, rank, world, spmm=oracle_spmm, rowops=NumpyRowOps)
        m.eval()
        g = torch.Generator().manual_seed(0)
        m.load_full_embedding(torch.randn(U + I + 2, d, generator=g) * 0.1)
        gr = torch.Generator().manual_seed(10 + rank)
        users = torch.randint(0, m.n_local, (B,), generator=gr)
        users[:3] = users[0]  # repeats
        items = torch.randint(0, I, (2 * B,), generator=gr)
        items[:4] = 7  # the same item on every rank
        G = torch.randn(3 * B, d, generator=gr)
        rep = m.batch_rep(users, items)
        (rep * G).sum().backward()
        m.sync_grads()
        q.put((rank, m.u0, m.u1, users.numpy(), items.numpy(), G.numpy(), rep.detach().numpy(),
               m.embedding.weight.grad.numpy()))
    except Exception:
        import traceback
        q.put((rank, 'error', traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,L', [(2, 1), (2, 3), (4, 2), (8, 3)])
def test_sharded_batch_rows_match_unsharded(world, L):
    """World 2, 4 and 8, last layer only at the batch rows: users local, items
    through the all-gathered item list and one small reduce; backward pulls +
    scattered terms."""
    rng = np.random.default_rng(5)
    U, I, d, B = 80, 60, 8, 12
    pairs = np.stack([rng.integers(0, U, 800), rng.integers(0, I, 800)], 1)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, pairs, U, I, d, L, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != 'error', r[2]
    A = O.norm_adj(U, I, pairs)
    F = O.generate_feat(U, I, pairs)
    fv = O.feat_values(F, 1.0)
    emb = (torch.randn(U + I + 2, d, generator=torch.Generator().manual_seed(0)) * 0.1).numpy()
    rep = O.igcn_rep(A, F, fv, emb, L)
    Gt = np.zeros((U + I, d), np.float32)
    for rank, u0, u1, users, items, G, _, _ in res:
        np.add.at(Gt, u0 + users, G[:B])
        np.add.at(Gt, U + items, G[B:])
    grad = O.igcn_grad(A, F, fv, L, Gt)
    tol = dict(rtol=1e-5, atol=1e-6)
    gtol = dict(rtol=1e-5, atol=1e-6 * max(1.0, float(np.abs(grad).max())))
    for rank, u0, u1, users, items, G, rep_b, grad_k in res:
        nk = u1 - u0
        np.testing.assert_allclose(rep_b, np.concatenate([rep[u0 + users], rep[U + items]]), **tol)
        np.testing.assert_allclose(grad_k[:nk], grad[u0:u1], **gtol)
        np.testing.assert_allclose(grad_k[nk:], grad[U:], **gtol)


def test_sharded_side_replicates_the_smaller_side():
    from igr.dist import sharded_side
    assert sharded_side(10_000_000, 1_000_000) == 'users'  # items replicated
    assert sharded_side(50_000, 2_900_000) == 'items'  # Amazon-Books-like: users replicated
    assert sharded_side(5, 10, 'items') == 'users' and sharded_side(10, 5, 'users') == 'items'
    with pytest.raises(ValueError):
        sharded_side(1, 1, 'both')


def test_swapped_sides_layer_matches_oracle():
    """With items outnumbering users the pairs are passed column-swapped (items sharded,
    users replicated); one layer then equals A x restricted to each side."""
    rng = np.random.default_rng(9)
    U, I, d = 30, 200, 8
    pairs = np.stack([rng.integers(0, U, 1500), rng.integers(0, I, 1500)], 1)
    sw = np.ascontiguousarray(pairs[:, ::-1])
    sh = BipartiteShard(sw, I, U, 0, 1, 'cpu')  # items are the cut side
    g = torch.Generator().manual_seed(1)
    x = torch.randn(U + I, d, generator=g)
    y_items, y_users = sh.layer(x[U:].contiguous(), x[:U].contiguous(), spmm=oracle_spmm)
    A = O.norm_adj(U, I, pairs)
    ref = O.spmm(A, x.numpy())
    np.testing.assert_allclose(y_users.numpy(), ref[:U], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(y_items.numpy(), ref[U:], rtol=1e-5, atol=1e-6)


# ------------------------------------------------------------------ rank-local set-up (BipartiteShard.from_stream)

def _stream_worker(rank, world, port, pairs, U, I, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        tm = {}
        a = BipartiteShard.from_stream(pairs[:, 0].copy(), pairs[:, 1].copy(), U, I, rank, world, 'cpu',
                                       timings=tm, item_tiles=2, item_chunks=2)
        b = BipartiteShard(pairs, U, I, rank, world, 'cpu', item_tiles=2, item_chunks=2)  # every rank counts everything
        same = (a.u0, a.u1) == (b.u0, b.u1) and np.array_equal(a.degree, b.degree) and a.local_nnz == b.local_nnz
        same = same and torch.equal(a.user_vals, b.user_vals)
        for k in ('row_ptr', 'col_idx'):
            same = same and np.array_equal(a.user_block.host()[k], b.user_block.host()[k])
        for k in ('row_ptr', 'col_idx', 'vals'):
            same = same and np.array_equal(a.item_host[k], b.item_host[k])
        for (r0, r1, ta), (s0, s1, tb) in zip(a.chunks, b.chunks):
            same = same and (r0, r1) == (s0, s1)
            for (ga, va, c0, c1), (gb, vb, e0, e1) in zip(ta, tb):
                same = same and (c0, c1) == (e0, e1) and torch.equal(va, vb)
                same = same and np.array_equal(ga.host()['col_idx'], gb.host()['col_idx'])
        q.put((rank, bool(same), sorted(tm), a.u0, a.u1, a.local_nnz))
    except Exception:
        import traceback
        q.put((rank, 'error', traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_from_stream_builds_the_same_shards(world):
    """Counting one slice of the stream per rank + a host all-reduce + a range select
    gives every rank exactly the shard the whole-list constructor builds."""
    U, I, E = 900, 200, 20000
    rng = np.random.default_rng(11)
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_worker, args=(r, world, port, pairs, U, I, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    errs = [r[2] for r in res if r[1] == 'error']
    assert not errs, errs[0]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = sorted(res)
    assert all(r[1] is True for r in res)
    assert res[0][2] == ['build_s', 'count_s', 'select_s']
    assert res[0][3] == 0 and res[-1][4] == U and all(a[4] == b[3] for a, b in zip(res, res[1:]))
    assert sum(r[5] for r in res) == O.norm_adj(U, I, pairs).nnz


def test_item_block_is_the_transposed_user_block():
    """Each source tile of the item block is built by transposing a range of user rows:
    together the tiles hold exactly the item rows of D^-1/2 A D^-1/2 (duplicate pairs summed)."""
    U, I, E = 500, 90, 6000
    rng = np.random.default_rng(3)
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)  # E >> U*I/8: many duplicate pairs
    A = O.norm_adj(U, I, pairs)
    dense = np.zeros((U + I, U + I), np.float32)
    rows = np.repeat(np.arange(U + I), np.diff(A.row_ptr))
    dense[rows, A.col] = A.val
    sh = BipartiteShard(pairs, U, I, 0, 1, 'cpu', item_tiles=3, item_chunks=2)
    got = np.zeros((I, U), np.float32)
    for r0, r1, tiles in sh.chunks:
        for g, v, c0, c1 in tiles:
            h = g.host()
            rr = np.repeat(np.arange(r0, r1), np.diff(h['row_ptr']))
            assert np.all(np.diff(h['row_ptr']) >= 0) and h['col_idx'].max(initial=0) < c1 - c0
            got[rr, h['col_idx'] + c0] = v.numpy()
    np.testing.assert_array_equal(got, dense[U:, :U])
    ih = sh.item_host
    full = np.zeros((I, U), np.float32)
    full[np.repeat(np.arange(I), np.diff(ih['row_ptr'])), ih['col_idx']] = ih['vals']
    np.testing.assert_array_equal(full, dense[U:, :U])
