"""Per-rank compute of bench.py's sharded layer at world 2 / 4 / 8, on one GPU.

The driver takes the real multi-GPU numbers; this measures what one rank's
SpMM launches cost at each partition of the default bench graph (10M users x
1M items, 200M draws, d=64), without the RCCL all-reduce: the compute floor
of the strong-scaling curve.  Every rank's shard is timed (they are balanced
by edge count; the slowest one sets the step).  Output: one JSON line.
"""
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
    ap.add_argument('--worlds', default='1,2,4,8')
    ap.add_argument('--d', type=int, default=64)
    ap.add_argument('--ranks', default='all', help="'all' or 'first'")
    ap.add_argument('--steps', type=int, default=10)
    args = ap.parse_args()
    from igr.dataset import synthetic_pairs
    from igr.dist import BipartiteShard
    dev = torch.device('cuda')
    U, I, E, d = 10_000_000, 1_000_000, 200_000_000, args.d
    su, si = synthetic_pairs(U, I, E, 0, stacked=False)
    from igr.graph import count_ids
    total = np.concatenate([count_ids(su, U), count_ids(si, I)])
    g = torch.Generator(device=dev).manual_seed(2)
    x_items = torch.randn(I, d, generator=g, device=dev) * 0.1
    out = {}
    for W in [int(w) for w in args.worlds.split(',')]:
        per = []
        for rank in (range(W) if args.ranks == 'all' else [0]):
            t0 = time.time()
            e0, e1 = E * rank // W, E * (rank + 1) // W
            others = total - np.concatenate([count_ids(su[e0:e1], U), count_ids(si[e0:e1], I)])
            shard = BipartiteShard.from_stream(su, si, U, I, rank, W, dev, d=d, reduce=lambda c, o=others: c + o)
            shard.exchange = False  # compute only: no collective
            nu = shard.u1 - shard.u0
            x_users = torch.randn(nu, d, generator=g, device=dev) * 0.1
            y_users = torch.empty(nu, d, device=dev)
            y_items = torch.empty(I, d, device=dev)
            for _ in range(3):
                shard.layer(x_users, x_items, y_users, y_items)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.steps):
                shard.layer(x_users, x_items, y_users, y_items)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.steps
            per.append({'rank': rank, 'ms': ms, 'local_nnz': shard.local_nnz, 'users': nu,
                        'item_tiles': shard.item_tiles, 'item_chunks': shard.item_chunks})
            print(f'W={W} rank {rank}: {ms:.3f} ms, local nnz {shard.local_nnz}, tiles {shard.item_tiles}, '
                  f'chunks {shard.item_chunks} (build {time.time() - t0:.1f}s)', file=sys.stderr, flush=True)
            del shard, x_users, y_users, y_items
            torch.cuda.empty_cache()
        worst = max(p['ms'] for p in per)
        out[f'w{W}'] = {'ranks': per, 'max_rank_ms': worst,
                        'compute_only_edges_per_s': sum(p['local_nnz'] for p in per) / worst * 1e3
                        if len(per) == W else None}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
