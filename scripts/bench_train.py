"""IGCN training-step throughput on one GPU (not the bench metric).

One step = IGCNTrainer.step: device BPR sampling (main + aux batch), dropout
of the feature values, inductive SpMM + L LightGCN SpMMs (fused layer mean),
fused BPR + aux losses, the backward (L reverse SpMMs + transposed feature
SpMM), fused Adam over the (N+2) x d table.  Synthetic uniform graph.
With batch_rep (default 'auto' -> taken here) the last forward layer and the
first backward layer run only at the 3B batch rows (ops.propagate_rows)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n-users', type=int, default=1_000_000)
    ap.add_argument('--n-items', type=int, default=100_000)
    ap.add_argument('--n-edges', type=int, default=20_000_000)
    ap.add_argument('--d', type=int, default=64)
    ap.add_argument('--layers', type=int, default=3)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=2048)
    ap.add_argument('--batch-rep', default='auto', choices=['auto', 'true', 'false'],
                    help='last layer only at the batch rows (model.batch_rep_pays)')
    ap.add_argument('--model', default='IGCN', choices=['IGCN', 'AttIGCN', 'LightGCN', 'NGCF', 'IMCGAE', 'IMF'])
    ap.add_argument('--l2-reg', type=float, default=0., help='trainer l2_reg (0 skips the l2 term, as the IGCN configs do)')
    ap.add_argument('--eval', action='store_true', help='also time one full eval ranking (Recall@20 path)')
    ap.add_argument('--graph', action='store_true', help='replay one hipGraph-captured step (trainer.StepGraph)')
    ap.add_argument('--epochs', type=int, default=0,
                    help='time this many train_one_epoch() calls of the trainer as configured by default (no '
                         "'graph' key: the trainer picks the captured step where it applies) instead of single steps")
    ap.add_argument('--dist-backend', default='nccl', help="'nccl' (= RCCL); 'gloo' for rehearsals (host-staged)")
    ap.add_argument('--one-device', action='store_true',
                    help='every rank on cuda:0 (multi-rank rehearsal on a one-GPU box, with --dist-backend gloo)')
    ap.add_argument('--sharded', action='store_true',
                    help='igr.dist_train.ShardedIGCN, one rank per GPU (per-rank batch --batch): under '
                         'torch.distributed.run, or with --gpus N this script starts the N ranks itself')
    ap.add_argument('--gpus', type=int, default=None,
                    help='ranks of the --sharded run (default: WORLD_SIZE when launched, else 1)')
    ap.add_argument('--item-dist', default='uniform', choices=['uniform', 'zipf'],
                    help='item popularity of the synthetic draws (zipf: exponent 1.1)')
    ap.add_argument('--skewed', default=None, metavar='SHAPE',
                    help="MovieLens-like item popularity: the training pairs of tests/golden/ml_like.py's SHAPE "
                         "('ml100k', 'ml1m', 'ml1m_l3', 'gowalla') instead of uniform draws (sets users / items / d / layers)")
    args = ap.parse_args()
    if args.sharded and args.gpus:
        from igr.launch import maybe_launch
        rc = maybe_launch(__file__, sys.argv[1:], args.gpus, one_device=args.one_device)
        if rc is not None:  # this process only started the ranks and waited for them
            sys.exit(rc)
    from igr import model as M
    from igr import trainer as T
    from igr.dataset import synthetic_pairs
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    assert not (args.sharded and args.gpus) or world == args.gpus, f'--gpus {args.gpus} but WORLD_SIZE={world}'
    if args.sharded and world > 1:
        import torch.distributed as dist
        local = 0 if args.one_device else int(os.environ.get('LOCAL_RANK', '0'))
        torch.cuda.set_device(local)
        if args.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(args.dist_backend)
    dev = torch.device('cuda')
    import threading
    building = threading.Event()

    def heartbeat():  # host-side setup of a 200M-edge graph takes minutes: keep the log moving
        t_hb = time.time()
        while not building.wait(30):
            print(f'... setting up ({time.time() - t_hb:.0f}s)', file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    if args.skewed:
        sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
        import ml_like
        args.n_users, args.n_items, mean_deg, args.d, args.layers, _ = ml_like.SHAPES[args.skewed]
        train, _, _ = ml_like.make_splits(args.n_users, args.n_items, mean_deg, seed=100)
        pairs = np.array([[u, i] for u in range(args.n_users) for i in train[u]], dtype=np.int64)
        args.n_edges = len(pairs)
    else:
        pairs = synthetic_pairs(args.n_users, args.n_items, args.n_edges, 0, args.item_dist)

    class DS:
        name = 'synthetic'
        n_users, n_items, train_pairs = args.n_users, args.n_items, pairs
        train_array = pairs
        train_data = None

        def __len__(self):
            return len(pairs)
    ds = DS()
    t0 = time.time()
    if args.sharded:
        return sharded(args, ds, rank, world, dev)
    if args.model == 'IMF':
        args.layers = 0  # the inductive layer alone (model.py:4290-4297)
    m = getattr(M, args.model)({'name': args.model, 'embedding_size': args.d, 'n_layers': args.layers,
                                'layer_sizes': [args.d] * args.layers,  # NGCF (config.py: [64, 64, 64])
                                'device': dev, 'dropout': 0.3 if args.model != 'NGCF' else 0.1, 'feature_ratio': 1.,
                                'dataset': ds,
                                'batch_rep': {'auto': 'auto', 'true': True, 'false': False}[args.batch_rep]})
    igcn = args.model in ('IGCN', 'AttIGCN', 'IMF')
    tr = T.get_trainer({'name': 'IGCNTrainer' if igcn else 'BPRTrainer', 'optimizer': 'Adam', 'lr': 1e-3,
                        'l2_reg': args.l2_reg, 'aux_reg': 0.01, 'device': dev, 'n_epochs': 1, 'batch_size': args.batch,
                        'test_batch_size': 512, 'topks': [20]}, ds, m)
    building.set()
    print(f'built in {time.time() - t0:.1f}s: adj nnz {m.norm_adj.nnz}' +
          (f', feat nnz {m.feat_mat.nnz}' if igcn else ''), file=sys.stderr, flush=True)
    m.train()

    def step():
        u, p, n = tr.sampler.sample(args.batch)
        if not igcn:
            return tr.step(u, p, n)
        au, ap_, an = tr.aux_sampler.sample(args.batch)
        return tr.step(u, p, n, au, ap_, an)
    if args.epochs:
        steps = len(tr.sampler)
        tr.train_one_epoch()  # builds the captured step (or not) and warms up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.epochs):
            loss = tr.train_one_epoch()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({'model': args.model, 'mode': 'train_one_epoch, default trainer config',
                          'captured_step': bool(T.graph_mode_for(tr)), 'steps_per_epoch': steps, 'epochs': args.epochs,
                          'epoch_s': el / args.epochs, 'ms_per_step': el / args.epochs / steps * 1e3, 'loss': float(loss),
                          'n_users': args.n_users, 'n_items': args.n_items, 'n_edges': args.n_edges, 'd': args.d,
                          'layers': args.layers}))
        return
    if args.graph:
        sg = T.StepGraph(tr, args.batch)

        def step():  # noqa: F811
            sg.replay()
            return sg.loss_sum
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    feat_nnz = m.feat_mat.nnz if igcn else 0
    if args.graph:
        loss = sg.take_loss() / ((args.steps + args.warmup + 2) * args.batch)
        sg.close()
    out = {'model': args.model, 'graph': args.graph, 'ms_per_step': el / args.steps * 1e3, 'loss': float(torch.as_tensor(loss).detach()),
           'n_users': args.n_users,
           'n_items': args.n_items, 'n_edges': args.n_edges, 'd': args.d, 'layers': args.layers,
           'adj_nnz': m.norm_adj.nnz, 'feat_nnz': feat_nnz,
           'batch_rep': M.batch_rep_pays(m, args.batch) if args.model == 'IGCN' or not igcn else False,
           'edges_per_s_fwd_bwd': (m.norm_adj.nnz * args.layers + feat_nnz) * 2 * args.steps / el}
    if args.eval:
        # one eval ranking over every user (rep once, MFMA scores, mask, top-k); no held-out lists in
        # the synthetic data, so the 'train' split (no exclusion) is timed
        tr.dataset.val_data = tr.dataset.test_data = None
        rec = tr.rank('train')  # warm-up (first-use allocations, code objects)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            rec = tr.rank('train')
        torch.cuda.synchronize()
        out['eval_rank_s'] = (time.perf_counter() - t0) / 3
        out['eval_users'] = int(rec.shape[0])
    print(json.dumps(out))


def sharded(args, ds, rank, world, dev):
    import torch.distributed as dist
    from igr.dist_train import ShardedIGCN, ShardedIGCNTrainer
    t0 = time.time()
    m = ShardedIGCN({'embedding_size': args.d, 'n_layers': args.layers, 'device': dev, 'dropout': 0.3,
                     'feature_ratio': 1., 'dataset': ds}, rank, world)
    tr = ShardedIGCNTrainer({'batch_size': args.batch, 'l2_reg': 0., 'aux_reg': 0.01, 'lr': 1e-3}, m)
    print(f'rank {rank}: built in {time.time() - t0:.1f}s: users [{m.u0}, {m.u1})', file=sys.stderr)
    m.train()
    for _ in range(args.warmup):
        tr.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = tr.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev if args.dist_backend == 'nccl' else 'cpu')  # gloo: CPU tensors only
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    if rank == 0:
        print(json.dumps({'mode': 'sharded', 'world': world, 'backend': args.dist_backend,
                          'one_device': args.one_device, 'ms_per_step': el / args.steps * 1e3,
                          'samples_per_s': world * args.batch * args.steps / el, 'loss': float(torch.as_tensor(loss).detach()),
                          'n_users': args.n_users, 'n_items': args.n_items, 'n_edges': args.n_edges, 'd': args.d,
                          'layers': args.layers}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
