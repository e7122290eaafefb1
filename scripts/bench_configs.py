"""One-GPU SpMM and forward numbers at the shapes of every BASELINE.json config.

For each config: a synthetic uniform bipartite graph of the dataset's shape
(public dataset statistics; the real interaction files are not in the image),
the symmetric D^-1/2 A D^-1/2 adjacency built exactly as
utils.generate_daj_mat + LightGCN.generate_graph (igr.model.build_norm_adj),
and
  * one SpMM Y = A X over the whole N x N adjacency (HIP events, median of 20
    launches after 3 warm-ups), with the algorithmic bytes
    nnz*(8 + 4d) + n*(8 + 4d) and their fraction of the 8 TB/s HBM peak.  Below
    ~100 MB of working set the tables live in L2 / Infinity Cache, so the
    fraction can exceed 1 there: it is not an HBM number at those sizes;
  * IGCN.get_rep (eval mode: feature SpMM + L adjacency SpMMs with the fused
    layer mean), eager and replayed from a hipGraph.
The synthetic 10M x 1M graph (configs[4], north star) is bench.py's workload
(`bench.py --d 64 / --d 256`), not repeated here.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBPS = 8000.0
# name: (users, items, interactions, d, layers, BASELINE config)
CONFIGS = {
    'ml100k': (943, 1682, 100_000, 32, 1, 'configs[0] MovieLens-100K, d=32, 1 layer'),
    'ml1m': (6040, 3706, 1_000_209, 64, 2, 'configs[1] MovieLens-1M, d=64, 2 layers'),
    'gowalla': (29_858, 40_981, 1_027_370, 128, 3, 'configs[2] Gowalla, d=128, 3 layers'),
    'amazon_book': (52_643, 91_599, 2_984_108, 128, 3,
                    'configs[3] Amazon-Book (LightGCN split statistics), d=128, per-GPU before sharding'),
}


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--only', nargs='*', default=None)
    args = ap.parse_args()
    from igr import model as M
    from igr import ops
    from igr.dataset import synthetic_pairs
    dev = torch.device('cuda')
    out = {}
    for name, (U, I, E, d, L, label) in CONFIGS.items():
        if args.only and name not in args.only:
            continue
        pairs = synthetic_pairs(U, I, E, 0)
        g, vals, _, _ = M.build_norm_adj(U, I, pairs, dev)
        n, nnz = g.n_rows, g.nnz
        x = torch.randn(n, d, device=dev) * 0.1
        y = torch.empty(n, d, device=dev)
        ms = timed(lambda: ops.spmm(g, x, vals, out=y))
        byts = nnz * (8 + 4 * d) + n * (8 + 4 * d)

        class DS:
            n_users, n_items, train_pairs = U, I, pairs
        m = M.get_model({'name': 'IGCN', 'embedding_size': d, 'n_layers': L, 'device': dev, 'dropout': 0.3,
                         'feature_ratio': 1.}, DS())
        m.eval()
        with torch.no_grad():
            eager = timed(lambda: m.get_rep())
            hg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(hg):
                m.get_rep()
            graphed = timed(lambda: hg.replay())
        fwd_edges = nnz * L + m.feat_mat.nnz
        out[name] = {'config': label, 'n_users': U, 'n_items': I, 'interactions': E, 'nnz_adj': nnz,
                     'nnz_feat': m.feat_mat.nnz, 'd': d, 'layers': L,
                     'spmm_ms': ms, 'spmm_edges_per_s': nnz / ms * 1e3,
                     'spmm_algorithmic_GBps': byts / ms / 1e6, 'spmm_frac_of_hbm_peak': byts / ms / 1e6 / HBM_PEAK_GBPS,
                     'working_set_MB': (nnz * 8 + n * (8 + 8 * d)) / 1e6,
                     'igcn_get_rep_ms_eager': eager, 'igcn_get_rep_ms_hipgraph': graphed,
                     'igcn_forward_edges_per_s': fwd_edges / min(eager, graphed) * 1e3}
        print(name, json.dumps(out[name]), file=sys.stderr, flush=True)
        del m, g, vals, x, y
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
