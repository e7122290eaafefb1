"""The inductive layer's SpMM (model.py:4184, 4189; timed separately from the adjacency).

IGCN's feature graph at feature_ratio = 1 over the synthetic bipartite graph
(rows [users; items], columns [user features; item features; 2 generals],
nnz = 2E + N) built by igr.dist_train.FeatureShard at world 1, with the
row-constant values row_sum ** -0.5 (alpha = 1).  Times, with HIP events per
launch, the forward x0 = F E (W_Scaled: no value array) without and with the
in-kernel dropout mask (keep 0.7), the reverse F^T dx with the column scale,
and the reverse with the scale folded into dx (the training backward's form).
Algorithmic bytes as bench.py (nnz (8 + 4d) + rows (8 + 4d)), which counts a
4-B value per edge that W_Scaled does not read."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n-users', type=int, default=10_000_000)
    ap.add_argument('--n-items', type=int, default=1_000_000)
    ap.add_argument('--n-edges', type=int, default=200_000_000)
    ap.add_argument('--d', type=int, default=64)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    args = ap.parse_args()
    from igr import ops
    from igr.dataset import synthetic_pairs
    from igr.dist_train import FeatureShard
    dev = torch.device('cuda')
    U, I, d = args.n_users, args.n_items, args.d
    t0 = time.time()
    pairs = synthetic_pairs(U, I, args.n_edges, 0)
    fs = FeatureShard(pairs, U, I, 0, U, 0, dev)
    del pairs
    g = fs.graph
    gr = g.reverse()
    print(f'built in {time.time() - t0:.1f}s: rows {g.n_rows}, cols {g.n_cols}, nnz {g.nnz}', file=sys.stderr)
    rv = fs.row_values(1.0)
    gen = torch.Generator(device=dev).manual_seed(2)
    emb = torch.randn(g.n_cols, d, device=dev, generator=gen) * 0.1
    dx = torch.randn(g.n_rows, d, device=dev, generator=gen) * 0.1
    out_f = torch.empty(g.n_rows, d, device=dev)
    out_r = torch.empty(g.n_cols, d, device=dev)
    cases = {
        'forward': lambda: ops.spmm_scaled(g, emb, ops.ScaledWeights(rv), out=out_f),
        'forward_dropout': lambda: ops.spmm_scaled(g, emb, ops.ScaledWeights(rv, None, 0.7, 5, 1), out=out_f),
        'reverse_col_scale': lambda: ops.spmm_scaled(gr, dx, ops.ScaledWeights(None, rv, 0.7, 5, 1, True), out=out_r),
        'reverse_prescaled': lambda: ops.spmm_scaled(gr, dx, ops.ScaledWeights(None, None, 0.7, 5, 1, True),
                                                     out=out_r),
    }
    res = {}
    for name, fn in cases.items():
        for _ in range(args.warmup):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        torch.cuda.synchronize()
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
        rows = g.n_rows if name.startswith('forward') else gr.n_rows
        byts = g.nnz * (8 + 4 * d) + rows * (8 + 4 * d)
        res[name] = {'ms': ms, 'edges_per_s': g.nnz / ms * 1e3, 'algorithmic_GBps': byts / ms / 1e6,
                     'frac': byts / ms / 1e6 / 8000.0}
    print(json.dumps({'graph': 'IGCN feature graph (feature_ratio 1)', 'n_users': U, 'n_items': I,
                      'n_draws': args.n_edges, 'nnz': g.nnz, 'd': d, 'launches': res}))


if __name__ == '__main__':
    main()
