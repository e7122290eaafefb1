"""Does the projection GEMM's time depend on how long the GPU has been busy?  Launches
Linear(64, 256) on 1.1 M rows back to back (pre-allocated C) and prints the per-launch HIP-event
times in blocks, next to a plain fill and a copy of the same C bytes (the write-side reference)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def times(fn, n):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    return np.array([e0.elapsed_time(e1) for e0, e1 in ev]) * 1e3


def main():
    from igr import _lib as L
    from igr.ops import _p, _stream
    dev = torch.device('cuda')
    m, n, k = int(os.environ.get('M', 1_100_002)), 256, 64
    a = torch.randn(m, k, device=dev)
    b = torch.randn(n, k, device=dev)
    c = torch.empty(m, n, device=dev)
    c2 = torch.randn(m, n, device=dev)

    def gemm():
        L.call('igr_gemm_f32', m, n, k, _p(a), k, 0, _p(b), k, 0, None, _p(c), n, None, 0, _stream())
    res = {'m': m}
    gemm()
    torch.cuda.synchronize()
    t = times(gemm, 600)
    res['gemm_us_blocks_of_50'] = [round(float(np.median(t[i:i + 50])), 1) for i in range(0, 600, 50)]
    res['gemm_us_first10'] = [round(float(x), 1) for x in t[:10]]
    res['gemm_us_min'] = float(t.min())
    t = times(lambda: c.fill_(1.0), 100)
    res['fill_us_median'] = float(np.median(t))
    t = times(lambda: c.copy_(c2), 100)
    res['copy_us_median'] = float(np.median(t))
    t = times(gemm, 100)
    res['gemm_us_after_copies'] = float(np.median(t))
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
