"""The sharded layer's ordering against a collective that really is asynchronous.

A one-rank RCCL all-reduce moves no data and gloo's staged path is synchronous, so neither
shows a missing stream dependency.  Here the exchange is replaced by a stand-in with the
stream semantics torch gives an RCCL collective - it runs on a stream of its own, which first
waits for the work already queued on the caller's stream; `wait()` makes the caller's stream
wait for it - that is slow (it spins for milliseconds before touching the data) and that
changes the data the way a second, identical rank would: partial sums are doubled.  Every
layer's result is then known exactly (doubling is exact in fp32):

    items' output = 2 x (A_iu x_u),   users' output = A_ui x_i   with x_i the doubled items

and any read before the exchange has finished, or an exchange started before its SpMM has
written, shows up as a wrong number.  The same stand-in with `wait()` switched off must give
different numbers: the check that the test can see a missing wait at all.
"""
import numpy as np
import pytest
import torch

from igr import comm, dist

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda')
SPIN = 20_000_000  # cycles the stand-in collective spins before it touches the data (milliseconds)


class _Work:
    def __init__(self, done, honour_wait):
        self.done, self.honour_wait = done, honour_wait

    def wait(self):
        if self.honour_wait:
            torch.cuda.current_stream().wait_event(self.done)
        return True


def _standin(side, honour_wait=True):
    def all_reduce_sum(t, group=None, async_op=False):
        cur = torch.cuda.current_stream()
        ready = torch.cuda.Event()
        ready.record(cur)                     # everything queued so far, the SpMM that wrote t included
        with torch.cuda.stream(side):
            side.wait_event(ready)
            torch.cuda._sleep(SPIN)
            t.mul_(2.0)                       # the sum over two identical ranks
            done = torch.cuda.Event()
            done.record(side)
        w = _Work(done, honour_wait)
        if async_op:
            return w
        w.wait()
        return None
    return all_reduce_sum


def _shard(chunks, tiles):
    rng = np.random.default_rng(2)
    U, I, E = 50_000, 8_000, 600_000
    sh = dist.BipartiteShard.from_stream(rng.integers(0, U, E), rng.integers(0, I, E), U, I, 0, 1, DEV,
                                         item_chunks=chunks, item_tiles=tiles)
    g = torch.Generator(device=DEV).manual_seed(0)
    return sh, torch.randn(U, 64, generator=g, device=DEV), torch.randn(I, 64, generator=g, device=DEV)


def _expected(sh, xu, xi, layers):
    """Chained layers with the items' output doubled after each one, no exchange involved."""
    assert sh.exchange is False
    for _ in range(layers):
        yu, yi = sh.layer(xu, xi)
        xu, xi = yu, yi * 2.0
    torch.cuda.synchronize()
    return xu, xi


@pytest.mark.parametrize('chunks,tiles', [(4, 1), (2, 3)])
def test_deferred_waits_order_the_layers_against_an_asynchronous_exchange(monkeypatch, chunks, tiles):
    sh, xu, xi = _shard(chunks, tiles)
    want_u, want_i = _expected(sh, xu, xi, 4)
    side = torch.cuda.Stream()
    monkeypatch.setattr(comm, 'all_reduce_sum', _standin(side))
    sh.exchange = True
    # chained layers, every wait deferred into the next layer (bench.py, propagate)
    got_u, got_i = sh.propagate(xu, xi, 4)
    torch.cuda.synchronize()
    assert torch.equal(got_u, want_u) and torch.equal(got_i, want_i)
    # single layers with the wait inside (dist_train), into fresh buffers and into the caller's
    yu, yi = sh.layer(xu, xi)
    torch.cuda.synchronize()
    sh.exchange = False
    pu, pi = sh.layer(xu, xi)
    assert torch.equal(yu, pu) and torch.equal(yi, pi * 2.0)


def test_a_missing_wait_is_visible_to_this_test(monkeypatch):
    """Sensitivity: with wait() doing nothing the next layer reads the items before the
    stand-in has doubled them, and the numbers differ."""
    sh, xu, xi = _shard(4, 1)
    want_u, want_i = _expected(sh, xu, xi, 3)
    side = torch.cuda.Stream()
    monkeypatch.setattr(comm, 'all_reduce_sum', _standin(side, honour_wait=False))
    sh.exchange = True
    got_u, got_i = sh.propagate(xu, xi, 3)
    torch.cuda.synchronize()
    side.synchronize()
    assert not torch.equal(got_u, want_u)


def _sync_standin():
    """The same arithmetic on the caller's own stream: ordered by construction."""
    def all_reduce_sum(t, group=None, async_op=False):
        t.mul_(2.0)
        return comm._Done() if async_op else None
    return all_reduce_sum


@pytest.mark.parametrize('layers', [0, 1, 3])
def test_sharded_igcn_forward_and_backward_are_ordered_against_an_asynchronous_exchange(monkeypatch, layers):
    """igr.dist_train.ShardedPropagate (full-layer path): the inductive layer's item rows are
    reduced while the first layer's item side runs, the layers' reduces are waited inside each
    layer, the backward reduces the batch items first.  One rank made to behave as one of two
    (model.world = 2, the exchange switched on); the run with the slow asynchronous stand-in must
    equal, bit for bit, the run whose stand-in works on the caller's own stream - representation
    and embedding gradient, in train mode (dropout drawn in the SpMM)."""
    from igr.dist_train import ShardedIGCN
    rng = np.random.default_rng(4)
    U, I, E, d = 20_000, 3_000, 200_000, 64
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)

    class DS:
        name, n_users, n_items, train_pairs = 'synthetic', U, I, pairs

    def run(standin):
        torch.manual_seed(0)
        m = ShardedIGCN({'embedding_size': d, 'n_layers': layers, 'device': DEV, 'dropout': 0.3, 'feature_ratio': 1.,
                         'dataset': DS(), 'batch_rep': False, 'seed': 5}, 0, 1)
        m.world, m.shard.exchange = 2, True  # one of two identical ranks, as far as the exchange goes
        monkeypatch.setattr(comm, 'all_reduce_sum', standin)
        m.train()
        rep = m.get_rep()
        g = torch.Generator(device=DEV).manual_seed(1)
        (rep * torch.randn(rep.shape, generator=g, device=DEV)).sum().backward()
        torch.cuda.synchronize()
        return rep.detach().clone(), m.embedding.weight.grad.detach().clone()

    want_rep, want_grad = run(_sync_standin())
    got_rep, got_grad = run(_standin(torch.cuda.Stream()))
    assert float(want_rep.abs().sum()) > 0 and float(want_grad.abs().sum()) > 0
    assert torch.equal(got_rep, want_rep)
    assert torch.equal(got_grad, want_grad)


@pytest.mark.parametrize('batch_rep', [True, False])
def test_sharded_training_steps_are_ordered_against_an_asynchronous_exchange(monkeypatch, batch_rep):
    """Three whole steps of ShardedIGCNTrainer (batch-row path and full-layer path: forward,
    backward, the gradient reduce, fused Adam) as one of two identical ranks - the all-gathers
    hand back this rank's data twice, the all-reduces double - with the slow asynchronous
    stand-in and with the one on the caller's own stream: every parameter bit for bit."""
    from igr.dist_train import ShardedIGCN, ShardedIGCNTrainer
    rng = np.random.default_rng(6)
    U, I, E, d = 20_000, 3_000, 200_000, 32
    pairs = np.stack([rng.integers(0, U, E), rng.integers(0, I, E)], 1)

    class DS:
        name, n_users, n_items, train_pairs = 'synthetic', U, I, pairs

    def gather_twice(out, t, group=None):
        out.copy_(torch.cat([t, t]).view(out.shape))
        return out

    def run(standin):
        torch.manual_seed(0)
        m = ShardedIGCN({'embedding_size': d, 'n_layers': 2, 'device': DEV, 'dropout': 0.3, 'feature_ratio': 1.,
                         'dataset': DS(), 'batch_rep': batch_rep, 'seed': 5}, 0, 1)
        tr = ShardedIGCNTrainer({'batch_size': 512, 'l2_reg': 1e-4, 'aux_reg': 0.01, 'lr': 1e-2, 'seed': 3}, m)
        m.world, m.shard.exchange = 2, True
        monkeypatch.setattr(comm, 'all_reduce_sum', standin)
        monkeypatch.setattr(comm, 'all_gather_into', gather_twice)
        m.train()
        losses = [float(tr.step().detach()) for _ in range(3)]
        torch.cuda.synchronize()
        return losses, {k: v.detach().clone() for k, v in m.state_dict().items()}

    want_l, want = run(_sync_standin())
    got_l, got = run(_standin(torch.cuda.Stream()))
    assert got_l == want_l and all(np.isfinite(want_l))
    for k in want:
        assert torch.equal(got[k], want[k]), k
