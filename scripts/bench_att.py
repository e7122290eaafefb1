"""The attention inductive layer's edge kernels at scale (model.py:4246-4275).

IGCN's feature graph over the synthetic bipartite graph (feature_ratio 1,
nnz_F = 2E + N, igr.dist_train.FeatureShard at world 1), H = 4 heads of d:
  sddmm      alpha[e, h] = <q[row_e, h, :], k[col_e, h, :]>      (igr_sddmm_dot_f32)
  softmax    per-row max-shifted exp / sum, head mean            (igr_att_softmax_f32)
  segment    gspmm copy_rhs max over alpha (the DGL-surface op)   (igr_segment_reduce_f32)
  spmm       out = SpMM(E, w) with the per-edge attention values (igr_spmm_f32)
HIP events per launch.  SDDMM algorithmic bytes:
nnz (8 + 2*4*H*d) + nnz * 4H (q row and k row per edge, no cache credit; the
kernel keeps a row's q in registers, so its compulsory bytes are
nnz (4 + 4*H*d + 4H) + rows * 4*H*d).  Softmax: 3 passes over the H scalars
of each edge + the write of w: nnz (4 + 3*4H + 4)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import torch  # noqa: E402


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n-users', type=int, default=10_000_000)
    ap.add_argument('--n-items', type=int, default=1_000_000)
    ap.add_argument('--n-edges', type=int, default=200_000_000)
    ap.add_argument('--d', type=int, default=64)
    ap.add_argument('--heads', type=int, default=4)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    args = ap.parse_args()
    from igr import ops
    from igr.dataset import synthetic_pairs
    from igr.dist_train import FeatureShard
    dev = torch.device('cuda')
    U, I, d, H = args.n_users, args.n_items, args.d, args.heads
    t0 = time.time()
    pairs = synthetic_pairs(U, I, args.n_edges, 0)
    fs = FeatureShard(pairs, U, I, 0, U, 0, dev)
    del pairs
    g = fs.graph
    print(f'built in {time.time() - t0:.1f}s: rows {g.n_rows}, cols {g.n_cols}, nnz {g.nnz}', file=sys.stderr)
    gen = torch.Generator(device=dev).manual_seed(3)
    q = torch.randn(g.n_rows, H * d, device=dev, generator=gen) * 0.1
    k = torch.randn(g.n_cols, H * d, device=dev, generator=gen) * 0.1
    emb = torch.randn(g.n_cols, d, device=dev, generator=gen) * 0.1
    alpha = torch.empty(g.nnz, H, device=dev)
    res = {}
    ms = timed(lambda: ops.sddmm_dot(g, q, k, H, out=alpha), args.steps, args.warmup)
    alg = g.nnz * (8 + 2 * 4 * H * d) + g.nnz * 4 * H
    comp = g.nnz * (4 + 4 * H * d + 4 * H) + g.n_rows * 4 * H * d
    res['sddmm'] = {'ms': ms, 'edges_per_s': g.nnz / ms * 1e3, 'algorithmic_GBps': alg / ms / 1e6,
                    'frac': alg / ms / 1e6 / 8000.0, 'compulsory_GBps': comp / ms / 1e6}
    # the folded form: one d-float source row per edge for all heads (igr_sddmm_shared_f32);
    # algorithmic bytes per edge: col + eid-free out row + one 4d-byte source row
    a2 = torch.empty_like(alpha)
    ms = timed(lambda: ops.sddmm_shared(g, q, emb, H, out=a2), args.steps, args.warmup)
    alg = g.nnz * (4 + 4 * d + 4 * H) + g.n_rows * (8 + 4 * H * d)
    res['sddmm_shared'] = {'ms': ms, 'edges_per_s': g.nnz / ms * 1e3, 'algorithmic_GBps': alg / ms / 1e6,
                           'frac': alg / ms / 1e6 / 8000.0}
    du = torch.empty(g.n_rows, H * d, device=dev)
    ms = timed(lambda: ops.spmm_shared_heads(g, emb, alpha, H, out=du), args.steps, args.warmup)
    res['spmm_shared_heads_bwd'] = {'ms': ms, 'edges_per_s': g.nnz / ms * 1e3, 'algorithmic_GBps': alg / ms / 1e6,
                                    'frac': alg / ms / 1e6 / 8000.0}
    del a2, du
    ms = timed(lambda: ops.segment_reduce(g, alpha, 'max'), args.steps, args.warmup)
    byts = g.nnz * 4 * H + g.n_rows * (8 + 4 * H)
    res['segment_max'] = {'ms': ms, 'edges_per_s': g.nnz / ms * 1e3, 'algorithmic_GBps': byts / ms / 1e6,
                          'frac': byts / ms / 1e6 / 8000.0}
    holder = {}

    def sm():
        holder['w'] = ops.att_softmax(g, alpha, ops.sqrt_scale(d))[0]
    ms = timed(sm, args.steps, args.warmup)
    byts = g.nnz * (4 + 3 * 4 * H + 4)
    res['softmax'] = {'ms': ms, 'edges_per_s': g.nnz / ms * 1e3, 'algorithmic_GBps': byts / ms / 1e6,
                      'frac': byts / ms / 1e6 / 8000.0}
    w = holder['w']
    out = torch.empty(g.n_rows, d, device=dev)
    ms = timed(lambda: ops.spmm(g, emb, w, out=out), args.steps, args.warmup)
    byts = g.nnz * (8 + 4 * d) + g.n_rows * (8 + 4 * d)
    res['spmm_att'] = {'ms': ms, 'edges_per_s': g.nnz / ms * 1e3, 'algorithmic_GBps': byts / ms / 1e6,
                       'frac': byts / ms / 1e6 / 8000.0}
    # its gradient with respect to E: the reverse-graph SpMM with the same per-edge weights, which
    # the reverse graph addresses through its edge ids - read in place (eid), or permuted once
    # into the reverse graph's order (perm) and then streamed (pos)
    rev = g.reverse()
    dy = torch.randn(g.n_rows, d, device=dev, generator=gen) * 0.1
    dx = torch.empty(g.n_cols, d, device=dev)
    ms_eid = timed(lambda: ops.spmm(rev, dy, w, out=dx), args.steps, args.warmup)
    ms_perm = timed(lambda: holder.__setitem__('p', w[rev.edge_id]), args.steps, args.warmup)
    ms_pos = timed(lambda: ops.spmm(rev.positional(), dy, holder['p'], out=dx), args.steps, args.warmup)
    res['spmm_att_bwd'] = {'ms_values_by_edge_id': ms_eid, 'ms_permute_values': ms_perm, 'ms_positional': ms_pos,
                           'frac_by_edge_id': byts / ms_eid / 1e6 / 8000.0,
                           'frac_permute_plus_positional': byts / (ms_perm + ms_pos) / 1e6 / 8000.0}
    print(json.dumps({'graph': 'IGCN feature graph (feature_ratio 1)', 'n_users': U, 'n_items': I,
                      'n_draws': args.n_edges, 'nnz': g.nnz, 'd': d, 'heads': H, 'launches': res}))


if __name__ == '__main__':
    main()
