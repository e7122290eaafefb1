"""Eval ranking cost breakdown (BasicTrainer.rank, trainer.py:146-182 of the reference):
score GEMM, train-item mask and top-k per user batch, on ML-1M / Gowalla shaped
synthetic graphs.  Prints per-stage milliseconds for the whole user set and one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

SHAPES = {'ml1m': (6040, 3706, 800_000, 64), 'gowalla': (29_858, 40_981, 1_027_370, 128)}


def timed(fn, reps=5):
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
    from igr import ops
    from igr.dataset import synthetic_pairs
    dev = torch.device('cuda')
    out = {}
    batches = [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else '512,4096').split(',')]
    for name, (U, I, E, d) in SHAPES.items():
        pairs = synthetic_pairs(U, I, E, 0)
        order = np.lexsort((pairs[:, 1], pairs[:, 0]))
        p = pairs[order]
        ptr = torch.from_numpy(np.searchsorted(p[:, 0], np.arange(U + 1)).astype(np.int64)).to(dev)
        cols = torch.from_numpy(p[:, 1].astype(np.int32)).to(dev)
        g = torch.Generator(device=dev).manual_seed(0)
        rep = torch.randn(U + I, d, generator=g, device=dev) * 0.1
        items = rep[U:]
        for B in batches:
            starts = list(range(0, U, B))

            def gemm_all():
                for s in starts:
                    ops.gemm(rep[s:min(U, s + B)], items)

            sc = [ops.gemm(rep[s:min(U, s + B)], items) for s in starts]

            def mask_all():
                for s, x in zip(starts, sc):
                    ops.mask_scores(x, ptr[s:s + x.shape[0] + 1], cols)

            def topk_all():
                for x in sc:
                    ops.topk(x, 100, values=False)

            t_g, t_m, t_k = timed(gemm_all), timed(mask_all), timed(topk_all)
            flops = 2.0 * U * I * d
            r = {'gemm_ms': t_g, 'mask_ms': t_m, 'topk_ms': t_k, 'total_ms': t_g + t_m + t_k,
                 'gemm_tflops': flops / t_g / 1e9, 'topk_GBps': U * I * 4 / t_k / 1e6}
            out[f'{name}_B{B}'] = r
            print(name, B, r, file=sys.stderr, flush=True)
            del sc
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
