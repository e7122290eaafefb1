"""Thread scaling of the CPU baselines on this host (the bench's cpu_baseline legs):
oracle/oracle.c orc_spmm_sum_f32 (OpenMP) and torch.sparse.mm(CSR) at d = 64 on a
bench-like sample (rows of ~20 random columns into a 1M x 64 table)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import igr_oracle as O  # noqa: E402


def main():
    lib = O.lib()
    rng = np.random.default_rng(0)
    R, nc, d = 500_000, 1_000_000, 64
    deg = rng.integers(10, 30, R)
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ci = rng.integers(0, nc, rp[-1]).astype(np.int64)
    v = rng.standard_normal(rp[-1]).astype(np.float32)
    x = rng.standard_normal((nc, d)).astype(np.float32)
    out = np.empty((R, d), np.float32)
    res = {'cpu_affinity': len(os.sched_getaffinity(0)), 'OMP_NUM_THREADS': os.environ.get('OMP_NUM_THREADS'),
           'edges': int(rp[-1]), 'port': {}, 'torch_sparse_mm': {}}
    for th in [1, 2, 4, 8, 16, 32]:
        lib.orc_spmm_sum_f32(R, d, rp, ci, v, None, x, d, out, d, th)
        t = time.perf_counter()
        n = 0
        while time.perf_counter() - t < 2.0:
            lib.orc_spmm_sum_f32(R, d, rp, ci, v, None, x, d, out, d, th)
            n += 1
        res['port'][th] = rp[-1] * n / (time.perf_counter() - t)
    A = torch.sparse_csr_tensor(torch.from_numpy(rp), torch.from_numpy(ci), torch.from_numpy(v), size=(R, nc))
    X = torch.from_numpy(x)
    for th in [1, 4, 16, 32]:
        torch.set_num_threads(th)
        torch.sparse.mm(A, X)
        t = time.perf_counter()
        n = 0
        while time.perf_counter() - t < 2.0:
            torch.sparse.mm(A, X)
            n += 1
        res['torch_sparse_mm'][th] = rp[-1] * n / (time.perf_counter() - t)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
