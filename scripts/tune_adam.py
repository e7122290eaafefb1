"""Fused Adam (igr_adam_f32) sweep: float4s per thread per trip (IGR_ADAM_U) x
grid cap (IGR_ADAM_GRID) x non-temporal traffic (IGR_ADAM_NT) on the training step's table (1.1 M x 64 fp32 =
70.4 M parameters, 28 B per parameter: p, g, m, v read, p, m, v written)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
import torch  # noqa: E402


def main():
    from igr import ops
    n = 1_100_002 * 64
    dev = torch.device('cuda')
    p, g, m, v = (torch.randn(n, device=dev) for _ in range(4))
    v.abs_()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {}
    # grid 16384 = the former cap; 0 = uncapped (one float4 per thread, the default)
    for U, grid, nt in [(1, 16384, 0), (1, 16384, 1), (1, 0, 0), (1, 0, 1), (2, 0, 1), (4, 0, 1), (2, 16384, 1),
                        (1, 32768, 0), (1, 32768, 1)]:
        if True:
            os.environ['IGR_ADAM_U'] = str(U)
            os.environ['IGR_ADAM_GRID'] = str(grid)
            os.environ['IGR_ADAM_NT'] = str(nt)

            def step():
                ops.L.call('igr_adam_f32', n, ops._p(p), ops._p(g), ops._p(m), ops._p(v), 1e-3, 0.9, 0.999, 1e-8,
                           0.0, 10, None, ops._stream())
            for _ in range(5):
                step()
            torch.cuda.synchronize()
            a.record()
            for _ in range(50):
                step()
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / 50 * 1e3
            out[f'U{U}_grid{grid}_nt{nt}'] = {'us': us, 'TBps': 28 * n / us / 1e6}
            print(U, grid, nt, f'{us:.1f} us', f'{28 * n / us / 1e6:.2f} TB/s', flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
