"""What the one-line drop-in (`import igr.dgl_compat as dgl`) costs next to the fused model:
the reference's own propagation sequence - graph from (column, row), L x gspmm mul/sum, stack,
mean (model.py:100-110) - forward and backward through the DGL-shaped surface, against
igr.ops.propagate (one fused pass per layer, layer mean in the SpMM epilogue).  HIP events."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    args = ap.parse_args()
    import igr.dgl_compat as dgl
    from igr import model as M
    from igr import ops
    from igr.dataset import synthetic_pairs
    dev = torch.device('cuda')
    shapes = {'ml1m': (6040, 3706, 1_000_209, 64, 2), 'gowalla': (29_858, 40_981, 1_027_370, 128, 3),
              '1m_x_100k': (1_000_000, 100_000, 20_000_000, 64, 3)}
    for name, (U, I, E, d, L) in shapes.items():
        pairs = synthetic_pairs(U, I, E, 0)

        class DS:
            n_users, n_items, train_pairs = U, I, pairs
        m = M.LightGCN({'name': 'LightGCN', 'embedding_size': d, 'n_layers': L, 'device': dev, 'dataset': DS()})
        g0 = m.norm_adj
        row = g0.edge_rows()
        column = torch.from_numpy(g0.host()['col_idx'].astype(np.int64)).to(dev)
        vals, n = m.norm_vals, U + I
        emb = m.embedding.weight
        G = torch.randn(n, d, device=dev)

        def dropin():
            emb.grad = None
            g = dgl.graph((column, row), num_nodes=n, device=dev)   # rebuilt per forward, as the reference does
            rep, layers = emb, [emb]
            for _ in range(L):
                rep = dgl.ops.gspmm(g, 'mul', 'sum', lhs_data=rep, rhs_data=vals)
                layers.append(rep)
            (torch.stack(layers, dim=0).mean(dim=0) * G).sum().backward()

        def fused():
            emb.grad = None
            (ops.propagate(m.norm_adj, emb, L, adj_vals=vals) * G).sum().backward()
        res = {'shape': name, 'n_users': U, 'n_items': I, 'nnz': g0.nnz, 'd': d, 'layers': L,
               'dropin_fwd_bwd_ms': timed(dropin, args.steps, args.warmup),
               'fused_fwd_bwd_ms': timed(fused, args.steps, args.warmup)}
        print(json.dumps(res), flush=True)
        del m, g0, row, column, vals, emb, G
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
