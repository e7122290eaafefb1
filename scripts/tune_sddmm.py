"""SDDMM variants (scripts/tune_sddmm.py build | run) at the feature-graph shapes of
the small configs and a mid-size graph.  `build` compiles one libigr variant per
macro set into inductive-recommendation_amd/variants/ (CPU side); `run` (GPU box)
times each variant in its own process (IGR_LIB) and prints one JSON line each."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'inductive-recommendation_amd')
VARIANTS = {
    'u4_split': '-DIGR_SDDMM_U=4 -DIGR_SDDMM_SPLIT=1',
    'u4_nosplit': '-DIGR_SDDMM_U=4 -DIGR_SDDMM_SPLIT=0',
    'u2_split': '-DIGR_SDDMM_U=2 -DIGR_SDDMM_SPLIT=1',
    'u2_nosplit': '-DIGR_SDDMM_U=2 -DIGR_SDDMM_SPLIT=0',
    'u1_split': '-DIGR_SDDMM_U=1 -DIGR_SDDMM_SPLIT=1',
}
SHAPES = {'ml1m': (6040, 3706, 1_000_209), 'gowalla': (29_858, 40_981, 1_027_370),
          'mid': (300_000, 100_000, 10_000_000)}


def build():
    sys.path.insert(0, PKG)
    import build as B
    base = list(B.CFLAGS)
    for name, flags in VARIANTS.items():
        B.CFLAGS = base + flags.split()
        B.build(lib=os.path.join(PKG, 'variants', f'libigr_{name}.so'), obj=os.path.join(PKG, 'build_v', name))
        print('built', name, flags)


def one(name):
    os.environ['IGR_LIB'] = os.path.join(PKG, 'variants', f'libigr_{name}.so')
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    from igr import model as M
    from igr import ops
    from igr.dataset import synthetic_pairs
    dev = torch.device('cuda')
    res = {'variant': name}
    for sh, (U, I, E) in SHAPES.items():
        pairs = synthetic_pairs(U, I, E, 0)

        class DS:
            n_users, n_items, train_pairs = U, I, pairs
        m = M.IGCN({'name': 'IGCN', 'embedding_size': 64, 'n_layers': 1, 'device': dev, 'dropout': 0.,
                    'feature_ratio': 1., 'dataset': DS()})
        g = m.feat_mat
        for h, d in [(4, 64), (1, 64)]:
            q = torch.randn(g.n_rows, h * d, device=dev)
            k = torch.randn(g.n_cols, h * d, device=dev)
            out = torch.empty(g.nnz * h, device=dev)
            for _ in range(3):
                ops.sddmm_dot(g, q, k, h, out=out)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for a, b in ev:
                a.record()
                ops.sddmm_dot(g, q, k, h, out=out)
                b.record()
            torch.cuda.synchronize()
            res[f'{sh}_h{h}_us'] = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
        del m, g
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    if sys.argv[1] == 'build':
        build()
    elif sys.argv[1] == 'run':
        for name in (sys.argv[2:] or VARIANTS):
            subprocess.run([sys.executable, __file__, 'one', name], check=True, timeout=300)
    else:
        one(sys.argv[2])
