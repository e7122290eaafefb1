"""Shared-source SDDMM variants (scripts/tune_att_shared.py build | run): edges per lane
group per trip and trips per pass, on IGCN's feature graph of the synthetic bipartite
graph (10 M x 1 M, nnz_F 411 M) at h = 4, d = 64.  `build` compiles one libigr per macro
set (CPU side); `run` times each in its own process (IGR_LIB), one JSON line each."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'inductive-recommendation_amd')
VARIANTS = {f'u{u}n{n}': f'-DIGR_SDDMM_SHARED_U={u} -DIGR_SDDMM_SHARED_NT={n}'
            for u, n in [(1, 8), (2, 3), (4, 1)]}
VARIANTS.update({f'g{u}': f'-DIGR_SPMM_SHARED_U={u}' for u in (1, 2, 8)})  # the gradient kernel's edges per group


def build():
    sys.path.insert(0, PKG)
    import build as B
    base = list(B.CFLAGS)
    for name, flags in VARIANTS.items():
        B.CFLAGS = base + flags.split()
        B.build(lib=os.path.join(PKG, 'variants', f'libigr_{name}.so'), obj=os.path.join(PKG, 'build_v', name))
        print('built', name, flags)


def one(name):
    if name != 'current':
        os.environ['IGR_LIB'] = os.path.join(PKG, 'variants', f'libigr_{name}.so')
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    from igr import ops
    from igr.dataset import synthetic_pairs
    from igr.dist_train import FeatureShard
    dev = torch.device('cuda')
    U, I, E = (int(os.environ.get(k, v)) for k, v in (('U', 10_000_000), ('I', 1_000_000), ('E', 200_000_000)))
    H, d = 4, 64
    pairs = synthetic_pairs(U, I, E, 0)
    g = FeatureShard(pairs, U, I, 0, U, 0, dev).graph
    del pairs
    gen = torch.Generator(device=dev).manual_seed(3)
    q = torch.randn(g.n_rows, H * d, device=dev, generator=gen) * 0.1
    emb = torch.randn(g.n_cols, d, device=dev, generator=gen) * 0.1
    out = torch.empty(g.nnz, H, device=dev)
    for _ in range(2):
        ops.sddmm_shared(g, q, emb, H, out=out)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(7)]
    for a, b in ev:
        a.record()
        ops.sddmm_shared(g, q, emb, H, out=out)
        b.record()
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    alg = g.nnz * (4 + 4 * d + 4 * H) + g.n_rows * (8 + 4 * H * d)
    du = torch.empty(g.n_rows, H * d, device=dev)
    for _ in range(2):
        ops.spmm_shared_heads(g, emb, out, H, out=du)
    torch.cuda.synchronize()
    for a, b in ev:
        a.record()
        ops.spmm_shared_heads(g, emb, out, H, out=du)
        b.record()
    torch.cuda.synchronize()
    ms2 = float(np.median([a.elapsed_time(b) for a, b in ev]))
    print(json.dumps({'variant': name, 'nnz': g.nnz, 'sddmm_shared_ms': ms, 'frac': alg / ms / 1e6 / 8000.0,
                      'spmm_shared_heads_ms': ms2, 'frac_bwd': alg / ms2 / 1e6 / 8000.0}), flush=True)


if __name__ == '__main__':
    if sys.argv[1] == 'build':
        build()
    elif sys.argv[1] == 'run':
        for name in (sys.argv[2:] or ['current'] + list(VARIANTS)):
            subprocess.run([sys.executable, __file__, 'one', name], check=True, timeout=300)
    else:
        one(sys.argv[2])
