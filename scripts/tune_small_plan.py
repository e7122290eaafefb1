"""Row-schedule sweep for the small BASELINE graphs (ML-1M, Gowalla shapes):
time one adjacency SpMM (norm_adj, HIP events over many replays) under
different (split_threshold, chunk_edges) plans.  A plan with chunk_edges
above the largest degree turns every row longer than split_threshold into a
single one-wave chunk (4 lane groups splitting its edges) plus a one-chunk
combine."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

SHAPES = {'ml1m': (6040, 3706, 1_000_000, 64), 'gowalla': (29_858, 40_981, 1_027_370, 128),
          'ml100k': (943, 1682, 100_000, 32)}
PLANS = [(512, 512), (64, 8192), (128, 8192), (256, 8192), (32, 8192), (64, 512), (128, 1024)]


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def skewed_pairs(shape):
    """The MovieLens-shaped (skewed item popularity) training pairs of the parity tests."""
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    import ml_like
    nu, ni, mean_deg, d, _L, _ = ml_like.SHAPES[shape]
    train, _, _ = ml_like.make_splits(nu, ni, mean_deg, seed=100)
    return nu, ni, d, np.array([[u, i] for u in range(nu) for i in train[u]], dtype=np.int64)


def main():
    from igr import graph as G, ops
    from igr.dataset import synthetic_pairs
    dev = torch.device('cuda')
    out = {}
    cases = {name: (U, I, d, synthetic_pairs(U, I, E, 0)) for name, (U, I, E, d) in SHAPES.items()}
    if '--skewed' in sys.argv:
        cases.update({'ml1m_skewed': skewed_pairs('ml1m_l3'), 'ml100k_skewed': skewed_pairs('ml100k'),
                      'gowalla_skewed': skewed_pairs('gowalla')})
        PLANS.extend([(256, 256), (128, 128), (128, 256), (256, 512), (64, 64), (64, 128), (384, 384), (192, 192),
                      (384, 512), (192, 384), (96, 192)])
    for name, (U, I, d, pairs) in cases.items():
        row = np.concatenate([pairs[:, 0], U + pairs[:, 1]])
        col = np.concatenate([U + pairs[:, 1], pairs[:, 0]])
        x = torch.randn(U + I, d, device=dev) * 0.1
        ref = None
        for st, ce in PLANS:
            g, v = G.Graph.from_coo(row, col, U + I, U + I, np.ones(len(row), np.float32), dedup=True, device=dev,
                                    split_threshold=st, chunk_edges=ce)
            v = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
            y = ops.spmm(g, x, v)
            if ref is None:
                ref = y.clone()
            err = float((y - ref).abs().max())
            us = timeit(lambda: ops.spmm(g, x, v, out=y))
            out[f'{name}_st{st}_ce{ce}'] = {'us': us, 'n_split': g.n_split, 'n_chunks': g.n_chunks, 'max_abs_diff': err}
            print(name, st, ce, f'{us:.1f} us', g.n_split, g.n_chunks, err, flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
