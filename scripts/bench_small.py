"""get_rep (forward propagation) latency on small graphs: eager vs hipGraph replay.

ML-1M / Gowalla / ML-100K-shaped synthetic graphs (BASELINE.json configs 0-2):
at these sizes a layer is tens of microseconds, so launch overhead matters;
the whole get_rep is captured once with torch.cuda.graph (every igr entry
point only enqueues on the current stream, so it is capture-safe)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

SHAPES = {'ml100k': (943, 1682, 80_000, 32, 1), 'ml1m': (6040, 3706, 800_000, 64, 2),
          'gowalla': (29_858, 40_981, 1_027_370, 128, 3)}


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    from igr import model as M
    from igr.dataset import synthetic_pairs
    dev = torch.device('cuda')
    out = {}
    for name, (U, I, E, d, L) in SHAPES.items():
        pairs = synthetic_pairs(U, I, E, 0)

        class DS:
            n_users, n_items, train_pairs = U, I, pairs
        for mname in ['LightGCN', 'IGCN']:
            m = M.get_model({'name': mname, 'embedding_size': d, 'n_layers': L, 'device': dev, 'dropout': 0.3,
                             'feature_ratio': 1.}, DS())
            m.eval()
            with torch.no_grad():
                eager = timeit(lambda: m.get_rep())
                m.get_rep()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    rep = m.get_rep()
                graphed = timeit(lambda: g.replay())
                ref = m.get_rep()
                g.replay()
                torch.cuda.synchronize()
                same = bool(torch.equal(ref, rep))
            nnz = m.norm_adj.nnz * L + (m.feat_mat.nnz if mname == 'IGCN' else 0)
            out[f'{name}_{mname}'] = {'eager_ms': eager, 'graph_ms': graphed, 'bitwise_equal_replay': same,
                                      'edges_per_s_graph': nnz / graphed * 1e3, 'd': d, 'L': L}
            print(name, mname, out[f'{name}_{mname}'], flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
