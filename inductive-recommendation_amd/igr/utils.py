"""igr.utils - the helpers of the reference's utils.py that its scripts and models
call by name: run set-up (`set_seed`, `init_run`, utils.py:13-30) and graph
construction (`generate_daj_mat`, `get_sparse_tensor`, `graph_rank_nodes`,
utils.py:33-50, 186-215), plus `AverageMeter` and `Unbuffered` (utils.py:280-305),
which code written against the reference imports by name (the trainers here
accumulate the epoch loss on the device and do not need a host-side meter)."""
import os
import random
import sys

import numpy as np
import torch


def set_seed(seed=0):
    """Seed every generator a run draws from: Python, numpy, torch (CPU and all devices)."""
    seed = int(seed)
    os.environ['PYTHONHASHSEED'] = str(seed)
    for seeder in (random.seed, np.random.seed, torch.manual_seed):
        seeder(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def init_run(log_path, seed):
    """Seed the run and send stdout / stderr to `log_path`/lo00gg.txt (the file name the
    reference uses), flushed at every line so a killed run keeps its log."""
    set_seed(seed)
    os.makedirs(log_path, exist_ok=True)
    log = open(os.path.join(log_path, 'lo00gg.txt'), 'w', buffering=1)
    sys.stdout = sys.stderr = log
    return log


def generate_daj_mat(dataset):
    """utils.py:42-50: the symmetric bipartite adjacency [[0, R], [R^T, 0]] of the
    training pairs as a scipy CSR matrix, duplicates summed - built by the
    library's C++ CSR builder (igr_csr_from_coo), not by scipy's."""
    import scipy.sparse as sp
    from .graph import csr_from_coo
    from .model import train_pairs
    pairs = train_pairs(dataset)
    U, n = dataset.n_users, dataset.n_users + dataset.n_items
    row = np.concatenate([pairs[:, 0], pairs[:, 1] + U])
    col = np.concatenate([pairs[:, 1] + U, pairs[:, 0]])
    rp, ci, v, _ = csr_from_coo(row, col, n, n, None, dedup=True, want_eid=False)
    return sp.csr_matrix((v, ci, rp), shape=(n, n), dtype=np.float32)


def get_sparse_tensor(mat, device):
    """utils.py:33-39: a scipy sparse matrix as the device object the models
    propagate over - here a Graph (CSR + schedule in HBM) carrying the float32
    values by edge id (`.values`), edge id = position in (row, col) order, the
    order of the reference's coalesced COO tensor."""
    from .graph import Graph, csr_from_coo
    coo = mat.tocoo()
    rp, ci, v, _ = csr_from_coo(coo.row, coo.col, mat.shape[0], mat.shape[1], coo.data.astype(np.float32),
                                dedup=True, want_eid=False)
    g = Graph(rp, ci, mat.shape[0], mat.shape[1], device=device)
    g.values = torch.from_numpy(v).to(device)
    return g


def graph_rank_nodes(dataset, ranking_metric):
    """utils.py:186-215 ('degree', 'sort' / 'greedy')."""
    from .model import graph_rank_nodes as rank
    return rank(dataset, ranking_metric)


class AverageMeter:
    """Running value / sum / count / average of a scalar (utils.py:280-295)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = self.avg = self.sum = self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


class Unbuffered:
    """Wraps a text stream so that every write reaches the file at once (utils.py:291-305):
    `sys.stdout = Unbuffered(sys.stdout)`.  Everything else is the wrapped stream's."""

    def __init__(self, stream):
        self.stream = stream

    def _through(self, method, payload):
        getattr(self.stream, method)(payload)
        self.stream.flush()

    def write(self, data):
        self._through('write', data)

    def writelines(self, datas):
        self._through('writelines', datas)

    def __getattr__(self, name):
        return getattr(self.stream, name)
