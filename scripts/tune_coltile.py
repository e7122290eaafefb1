"""Column (feature) slicing of the wide-row SpMM on the bench graph: at d = 128 / 256
the item table (1M x d floats) outgrows the 256 MB Infinity Cache, so the
user-side gathers fall to HBM random-row rates; W passes over d/W-column slices
each gather from an (I x W)-float slice that fits.  Times one launch vs W-column
slices for each side (HIP events, median of 5)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))


def main():
    import numpy as np
    import torch
    from igr import ops
    from igr.dataset import synthetic_pairs
    from igr.dist import BipartiteShard
    dev = torch.device('cuda')
    U, I, E = 10_000_000, 1_000_000, 200_000_000
    pairs = synthetic_pairs(U, I, E, 0)
    sh = BipartiteShard(pairs, U, I, 0, 1, dev, item_tiles=1, item_chunks=1)
    del pairs
    out = {}

    def timeit(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    for d in (128, 256):
        xi = torch.randn(I, d, device=dev)
        xu = torch.randn(U, d, device=dev)
        yu = torch.empty(U, d, device=dev)
        yi = torch.empty(I, d, device=dev)
        for W in (d, 128, 64, 32):
            if W > d:
                continue

            def user():
                for c in range(0, d, W):
                    ops.spmm(sh.user_block, xi[:, c:c + W], sh.user_vals, out=yu[:, c:c + W])

            def item():
                for c in range(0, d, W):
                    ops.spmm(sh.item_block, xu[:, c:c + W], sh.item_vals, out=yi[:, c:c + W])
            out[f'd{d}_user_W{W}_ms'] = timeit(user)
            out[f'd{d}_item_W{W}_ms'] = timeit(item)
            print(d, W, out[f'd{d}_user_W{W}_ms'], out[f'd{d}_item_W{W}_ms'], file=sys.stderr, flush=True)
        del xi, xu, yu, yi
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
