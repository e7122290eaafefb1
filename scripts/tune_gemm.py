"""MFMA GEMM variants (scripts/tune_gemm.py build | run): the AttIGCN / NGCF
projection shapes at ML-1M and synthetic scale, their weight gradients (split-K)
and the eval score GEMM (users x d by items x d).  `build` compiles one libigr
per macro set (CPU side); `run` times each in its own process (IGR_LIB)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'inductive-recommendation_amd')
VARIANTS = {
    # the store placement of the persistent projection kernel
    'p_pin0': '-DIGR_GEMMP_PIN=0',                          # nothing may cross a store
    # diagnostics: what it costs to store C / load A
    'p_nostore': '-DIGR_GEMMP_NOSTORE',
    # k steps per load group of the streamed weight-gradient kernel
    'wg_pf4_w2048': '-DIGR_WGRAD_PF=4 -DIGR_WGRAD_OCC=2 -DIGR_WGRAD_WAVES=2048',
    'wg_pf12_w1024': '-DIGR_WGRAD_PF=12',
}
# the streamed Linear weight / bias gradient (m, n_out, k_in): timed next to the split-K GEMM + column sum it replaces
WGRAD = {'wgrad_att_ml1m': (9748, 256, 64), 'wgrad_att_1m': (1_100_002, 256, 64), 'wgrad_ngcf_1m': (1_100_000, 64, 64),
         'wgrad_att_11m': (11_000_002, 256, 64)}
ONLY = os.environ.get('IGR_TUNE_SHAPES')
# name: (m, n, k, trans_a, trans_b)
SHAPES = {
    'att_fwd_ml1m': (9748, 256, 64, False, False), 'att_dx_ml1m': (9748, 64, 256, False, True),
    'att_dw_ml1m': (256, 64, 9748, True, True),
    'att_fwd_1m': (1_100_002, 256, 64, False, False), 'att_dw_1m': (256, 64, 1_100_002, True, True),
    'ngcf_fwd_1m': (1_100_000, 64, 64, False, False), 'att_fwd_d32_1m': (1_100_002, 128, 32, False, False),
    'att_fwd_11m': (11_000_002, 256, 64, False, False),
    'score_gowalla': (4096, 40981, 128, False, False), 'score_ml1m': (6040, 3706, 64, False, False),
}


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
    dev = torch.device('cuda')
    res = {'variant': name}
    for sh, (m, n, k, ta, tb) in SHAPES.items():
        if ONLY and sh not in ONLY.split(','):
            continue
        a = torch.randn(*((k, m) if ta else (m, k)), device=dev)
        b = torch.randn(*((k, n) if tb else (n, k)), device=dev)
        # The first ~50 launches after an idle GPU run 10-30 % slower than the sustained rate
        # (clock / power management settling; scripts/gemm_clock_probe.py), so: `cold_us` = median
        # of the first 20 launches after 3, `us` = median of 50 launches after >= 150 ms of them.
        def timed(cnt):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(cnt)]
            for e0, e1 in ev:
                e0.record()
                ops.gemm(a, b, trans_a=ta, trans_b=tb)
                e1.record()
            torch.cuda.synchronize()
            return [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
        for _ in range(3):
            c = ops.gemm(a, b, trans_a=ta, trans_b=tb)
        torch.cuda.synchronize()
        cold = timed(20)
        n_warm = int(min(2000, max(20, 150e3 / max(float(np.median(cold)), 1.0))))
        timed(n_warm)
        us = float(np.median(timed(50)))
        ref = (a.t() if ta else a).double() @ (b if tb else b.t()).double()
        err = float(((c.double() - ref).abs().max() / ref.abs().max()).item())
        res[sh] = {'us': us, 'cold_us': float(np.median(cold)), 'tflops': 2 * m * n * k / us / 1e6, 'max_rel_err': err}
        del a, b, c, ref
        torch.cuda.empty_cache()
    for sh, (m, n, k) in WGRAD.items():
        if ONLY and sh not in ONLY.split(','):
            continue
        dy = torch.randn(m, n, device=dev)
        x = torch.randn(m, k, device=dev)

        def run(fn, cnt):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(cnt)]
            for e0, e1 in ev:
                e0.record()
                fn()
                e1.record()
            torch.cuda.synchronize()
            return float(np.median([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]))
        old = lambda: (ops.gemm(dy, x, trans_a=True, trans_b=True), dy.sum(0))  # noqa: E731
        new = lambda: ops.linear_wgrad(dy, x)  # noqa: E731
        out = {}
        for name_, fn in (('gemm_plus_sum_us', old), ('streamed_us', new)):
            run(fn, 10)
            run(fn, int(min(500, max(10, 100e3 / max(run(fn, 5), 1.0)))))
            out[name_] = run(fn, 30)
        out['bytes'] = 4 * m * (n + k)
        out['streamed_GBps'] = out['bytes'] / out['streamed_us'] / 1e3
        out['streamed_tflops'] = 2 * m * n * k / out['streamed_us'] / 1e6
        res[sh] = out
        del dy, x
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    if sys.argv[1] == 'build':
        build()
    elif sys.argv[1] == 'run':
        for name in (sys.argv[2:] or ['current'] + list(VARIANTS)):
            subprocess.run([sys.executable, __file__, 'one', name], check=True, timeout=300)
    else:
        one(sys.argv[2])
