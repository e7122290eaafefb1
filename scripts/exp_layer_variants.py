"""One propagation layer of the bench graph, three ways (timing experiment, one GPU):
  tiled      the shard layer as bench.py runs it: item-side source tiles, then the user side
  streams    the same launches with the item side and the user side on two streams
  whole      ONE launch over the whole symmetric adjacency [users; items] (the model's graph)
Prints ms per layer and G edges/s for each; checks that all three agree."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def timeit(fn, n=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n-users', type=int, default=10_000_000)
    ap.add_argument('--n-items', type=int, default=1_000_000)
    ap.add_argument('--n-edges', type=int, default=200_000_000)
    ap.add_argument('--d', type=int, default=64)
    ap.add_argument('--windows', default='65536')
    args = ap.parse_args()
    from igr import ops
    from igr.dataset import synthetic_pairs
    from igr.dist import BipartiteShard
    from igr.graph import Graph, csr_from_coo, sym_norm_values
    dev = torch.device('cuda')
    U, I, E, d = args.n_users, args.n_items, args.n_edges, args.d
    u, i = synthetic_pairs(U, I, E, 0, stacked=False)
    sh = BipartiteShard.from_stream(u, i, U, I, 0, 1, dev, d=d)
    nnz = sh.local_nnz
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn(U + I, d, generator=g, device=dev) * 0.1
    xu, xi = x[:U], x[U:]
    y = torch.empty_like(x)
    yu, yi = y[:U], y[U:]
    out = {'nnz': nnz, 'd': d}
    out['tiled_ms'] = timeit(lambda: sh.layer(xu, xi, yu, yi))
    ref = y.clone()
    side = torch.cuda.Stream()

    def streams():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for r0, r1, tiles in sh.chunks:
                for t, (gt, v, c0, c1) in enumerate(tiles):
                    if t == 0:
                        ops.spmm(gt, xu[c0:c1], v, out=yi[r0:r1])
                    else:
                        ops.spmm(gt, xu[c0:c1], v, out=yi[r0:r1], epi=ops.epilogue(beta=1.0, add=yi[r0:r1]))
        ops.spmm(sh.user_block, xi, sh.user_vals, out=yu)
        cur.wait_stream(side)
    out['streams_ms'] = timeit(streams)
    assert torch.equal(y, ref)
    # the whole symmetric adjacency as one CSR: rows [users; items]
    ub, ih = sh.user_block.host(), sh.item_host
    rp = np.concatenate([ub['row_ptr'], ih['row_ptr'][1:] + ub['row_ptr'][-1]])
    ci = np.concatenate([ub['col_idx'] + np.int32(U), ih['col_idx']])
    vals = torch.cat([sh.user_vals, torch.from_numpy(ih['vals']).to(dev)])
    for w in [int(s) for s in args.windows.split(',')]:
        gw = Graph(rp, ci, U + I, U + I, device=dev, window=w)
        y.zero_()
        out[f'whole_w{w}_ms'] = timeit(lambda: ops.spmm(gw, x, vals, out=y))
        # item rows may differ from the tiled path in the last bit (tiles add partial sums)
        err = float((y - ref).abs().max() / ref.abs().max())
        assert err < 1e-5, err
        del gw
    # the two sides as two launches over the whole table (no tiles), one stream
    gi = Graph(ih['row_ptr'], ih['col_idx'], I, U, device=dev)
    iv = torch.from_numpy(ih['vals']).to(dev)
    out['item_untiled_ms'] = timeit(lambda: ops.spmm(gi, xu, iv, out=yi))
    out['user_ms'] = timeit(lambda: ops.spmm(sh.user_block, xi, sh.user_vals, out=yu))
    for k in list(out):
        if k.endswith('_ms') and k not in ('item_untiled_ms', 'user_ms'):
            out[k.replace('_ms', '_Gedges')] = nnz / out[k] / 1e6
    print(json.dumps(out))


if __name__ == '__main__':
    main()
