"""Sharded IGCN training (igr/dist_train.py) on the GPU against the single-GPU
model / trainer.

* world 1: ShardedIGCNTrainer == IGCNTrainer step for step (same init, same
  batches, dropout 0): losses and parameters after every Adam step.
* world 2 on ONE GPU (two processes, gloo over HIP tensors - RCCL refuses two
  ranks on one device): the ranks' steps equal a single-GPU model stepping on
  the mean of the two ranks' losses (each rank's batch in global ids).
Tolerance: 1e-5 relative (+1e-6 absolute) - fp32 reassociation only."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from igr import model as M
from igr import trainer as T

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda')
U, I, D, L, B, STEPS = 400, 300, 32, 2, 256, 3


class DS:
    name = 'synthetic'

    def __init__(self, pairs):
        self.train_pairs, self.n_users, self.n_items = pairs, U, I
        self.train_array = pairs

    def __len__(self):
        return len(self.train_pairs)


def _pairs():
    rng = np.random.default_rng(8)
    p = np.stack([rng.integers(0, U, 6000), rng.integers(0, I, 6000)], 1)
    return np.concatenate([p, p[:50]])


def _cfg(ds):
    return {'name': 'IGCN', 'embedding_size': D, 'n_layers': L, 'device': DEV, 'dropout': 0., 'feature_ratio': 1.,
            'dataset': ds, 'batch_rep': False}


def _batches(seed, lo, hi):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(STEPS):
        out.append(tuple(rng.integers(a, b, B) for a, b in [(lo, hi), (0, I), (0, I), (lo, hi), (0, I), (0, I)]))
    return out


def _single(pairs, emb0, batch_lists):
    """Single-GPU IGCN: the loss of step s is the mean over the batch lists of the trainer terms."""
    m = M.IGCN(_cfg(DS(pairs)))
    with torch.no_grad():
        m.embedding.weight.copy_(emb0)
    from igr.optim import Adam
    opt = Adam(m.parameters(), lr=1e-3)
    m.train()
    losses = []
    for s in range(STEPS):
        tot = 0.
        for bl in batch_lists:
            u, p, n, au, ap, an = (torch.from_numpy(a).to(DEV) for a in bl[s])
            bpr, l2, aux = m.bpr_aux_loss(u, p, n, au, ap, an)
            tot = tot + (bpr + 1e-4 * l2 + 0.01 * aux) / len(batch_lists)
        opt.zero_grad()
        tot.backward()
        opt.step()
        losses.append(float(tot.detach()))
    return losses, m.embedding.weight.detach().cpu().numpy(), m.w.detach().cpu().numpy()


@pytest.mark.parametrize('batch_rep', [False, True])
def test_sharded_world1_equals_igcn_trainer(batch_rep):
    from igr.dist_train import ShardedIGCN, ShardedIGCNTrainer
    pairs = _pairs()
    torch.manual_seed(0)
    emb0 = torch.randn(U + I + 2, D) * 0.1
    bl = _batches(1, 0, U)
    ref_losses, ref_emb, ref_w = _single(pairs, emb0.to(DEV), [bl])
    m = ShardedIGCN(dict(_cfg(DS(pairs)), batch_rep=batch_rep), 0, 1)
    assert m.batch_rows is batch_rep
    m.load_full_embedding(emb0)
    tr = ShardedIGCNTrainer({'batch_size': B, 'l2_reg': 1e-4, 'aux_reg': 0.01, 'lr': 1e-3}, m)
    m.train()
    for s in range(STEPS):
        loss = tr.step(*(torch.from_numpy(a).to(DEV) for a in bl[s]))
        assert float(loss.detach()) == pytest.approx(ref_losses[s], rel=1e-5)
    np.testing.assert_allclose(m.embedding.weight.detach().cpu().numpy(), ref_emb, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(m.w.detach().cpu().numpy(), ref_w, rtol=1e-5, atol=1e-6)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, pairs, emb0, q, batch_rep):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from igr.dist_train import ShardedIGCN, ShardedIGCNTrainer
        dev = torch.device('cuda')
        cfg = dict(_cfg(DS(pairs)), batch_rep=batch_rep)
        m = ShardedIGCN(cfg, rank, world)
        m.load_full_embedding(emb0)
        tr = ShardedIGCNTrainer({'batch_size': B, 'l2_reg': 1e-4, 'aux_reg': 0.01, 'lr': 1e-3}, m)
        m.train()
        bl = _batches(10 + rank, m.u0, m.u1)
        losses = []
        for s in range(STEPS):
            u, p, n, au, ap, an = (torch.from_numpy(a).to(dev) for a in bl[s])
            loss = tr.step(u - m.u0, p, n, au - m.u0, ap, an)  # local user ids
            losses.append(float(loss))
        q.put((rank, m.u0, m.u1, losses, m.embedding.weight.detach().cpu().numpy(), m.w.detach().cpu().numpy()))
    except Exception:
        import traceback
        q.put((rank, 'error', traceback.format_exc(), None, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('batch_rep', [False, True])
def test_sharded_world2_one_gpu_equals_single_gpu(batch_rep):
    pairs = _pairs()
    torch.manual_seed(0)
    emb0 = torch.randn(U + I + 2, D) * 0.1
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, pairs, emb0, q, batch_rep)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
    for r in res:
        assert r[1] != 'error', r[2]
    bls = [_batches(10 + r[0], r[1], r[2]) for r in res]
    ref_losses, ref_emb, ref_w = _single(pairs, emb0.to(DEV), bls)
    for s in range(STEPS):  # the global loss is the mean of the ranks' losses
        assert np.mean([r[3][s] for r in res]) == pytest.approx(ref_losses[s], rel=1e-5)
    for rank, u0, u1, _, emb, w in res:
        nk = u1 - u0
        np.testing.assert_allclose(emb[:nk], ref_emb[u0:u1], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(emb[nk:], ref_emb[U:], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(w, ref_w, rtol=1e-5, atol=1e-6)
