"""Rank-local set-up of the sharded bench graph: seconds per stage for rank r of world w,
measured for ONE rank at a time with the box's whole CPU share (on a multi-GPU node every
rank has its own cores; ranks rehearsing on a one-GPU box share 16, which hides the scaling).
The degree all-reduce is replaced by adding the other slices' counts, computed outside the
timed region.  Prints one JSON line: world -> stages of rank 0 and of the last rank."""
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
    ap.add_argument('--n-users', type=int, default=10_000_000)
    ap.add_argument('--n-items', type=int, default=1_000_000)
    ap.add_argument('--n-edges', type=int, default=200_000_000)
    ap.add_argument('--worlds', default='1,2,4,8')
    ap.add_argument('--device', default='cuda')
    args = ap.parse_args()
    from igr.dataset import synthetic_pairs
    from igr.dist import BipartiteShard
    from igr.graph import count_ids
    U, I, E = args.n_users, args.n_items, args.n_edges
    t0 = time.perf_counter()
    u, i = synthetic_pairs(U, I, E, 0, stacked=False)
    draw_s = time.perf_counter() - t0
    total = np.concatenate([count_ids(u, U), count_ids(i, I)])
    out = {'n_users': U, 'n_items': I, 'n_draws': E, 'draw_s': round(draw_s, 3), 'device': args.device,
           'threads': int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or len(os.sched_getaffinity(0)), 'worlds': {}}
    for w in [int(x) for x in args.worlds.split(',')]:
        res = {}
        for rank in sorted({0, w - 1}):
            e0, e1 = E * rank // w, E * (rank + 1) // w
            others = total - np.concatenate([count_ids(u[e0:e1], U), count_ids(i[e0:e1], I)])
            tm = {}
            t0 = time.perf_counter()
            sh = BipartiteShard.from_stream(u, i, U, I, rank, w, args.device, timings=tm,
                                            reduce=lambda c, o=others: c + o)
            if args.device != 'cpu':
                torch.cuda.synchronize()
            tm['total_s'] = time.perf_counter() - t0
            tm['local_nnz'] = sh.local_nnz
            res[f'rank{rank}'] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in tm.items()}
            del sh
        out['worlds'][str(w)] = res
    w1 = out['worlds'].get('1', {}).get('rank0', {}).get('total_s')
    if w1:
        out['ratio_to_ideal'] = {w: round(max(r['total_s'] for r in res.values()) / (w1 / int(w)), 2)
                                 for w, res in out['worlds'].items()}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
