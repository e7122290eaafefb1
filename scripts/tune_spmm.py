"""Timing experiments for the SpMM on the bench graph (run on the GPU box).

  python scripts/tune_spmm.py --variants default,u4w8,...   (spawns one process per library variant)
  python scripts/tune_spmm.py --lib PATH                     (one variant: windows x tilings)
Variant libraries are built by scripts/build_variants.sh into inductive-recommendation_amd/variants/."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def timeit(fn, reps=10):
    import numpy as np
    import torch
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def one(args):
    if args.lib:
        os.environ['IGR_LIB'] = args.lib
    sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
    import torch
    from igr import graph as G
    from igr import ops
    from igr.dataset import synthetic_pairs
    from igr.dist import BipartiteShard
    U, I, E, d = args.n_users, args.n_items, args.n_edges, args.d
    dev = torch.device('cuda')
    pairs = synthetic_pairs(U, I, E, 0, args.item_dist)
    res = {'lib': args.lib or 'default'}
    g = torch.Generator(device=dev).manual_seed(2)
    xi = torch.randn(I, d, generator=g, device=dev) * 0.1
    xu = torch.randn(U, d, generator=g, device=dev) * 0.1
    yi = torch.empty(I, d, device=dev)
    yu = torch.empty(U, d, device=dev)
    for window in [int(w) for w in args.windows.split(',')]:
        G.DEFAULT_WINDOW = window
        sh = BipartiteShard(pairs, U, I, 0, 1, dev)
        res[f'w{window}_item'] = timeit(lambda: ops.spmm(sh.item_block, xu, sh.item_vals, out=yi))
        res[f'w{window}_user'] = timeit(lambda: ops.spmm(sh.user_block, xi, sh.user_vals, out=yu))
        for T in [int(t) for t in args.tiles.split(',') if t]:
            b = [int(round(k * U / T)) for k in range(T + 1)]
            tg = G.TiledGraph(sh.item_block.host(), I, U, b, dev)
            tv = tg.tile_values(sh.item_vals)
            res[f'w{window}_item_T{T}'] = timeit(lambda: ops.spmm_tiled(tg, xu, tv, out=yi))
            del tg, tv
        del sh
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', default=None)
    ap.add_argument('--variants', default=None)
    ap.add_argument('--windows', default='0,65536')
    ap.add_argument('--tiles', default='4')
    ap.add_argument('--n-users', type=int, default=10_000_000)
    ap.add_argument('--n-items', type=int, default=1_000_000)
    ap.add_argument('--n-edges', type=int, default=200_000_000)
    ap.add_argument('--d', type=int, default=64)
    ap.add_argument('--item-dist', default='uniform')
    args = ap.parse_args()
    if args.variants:
        for v in args.variants.split(','):
            lib = '' if v == 'default' else os.path.join(ROOT, 'inductive-recommendation_amd', 'variants', v, 'libigr.so')
            cmd = [sys.executable, __file__, '--windows', args.windows, '--tiles', args.tiles, '--d', str(args.d),
                   '--n-users', str(args.n_users), '--n-items', str(args.n_items), '--n-edges', str(args.n_edges),
                   '--item-dist', args.item_dist] + (['--lib', lib] if lib else [])
            t0 = time.time()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            print(v, r.stdout.strip() or r.stderr[-2000:], f'({time.time() - t0:.0f}s)', flush=True)
            if r.returncode != 0:
                break
    else:
        one(args)


if __name__ == '__main__':
    main()
