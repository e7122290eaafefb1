"""igr.sampler - device-side BPR negative sampler (igr_bpr_sample).

Same distribution as BasicDataset.__getitem__ (dataset.py:119-131): a user
uniform over users with training items, a positive uniform over that user's
items, a negative uniform over items not in the user's training list.  The
training lists live in HBM as a CSR; each batch is one kernel launch with a
counter-based RNG keyed by (seed, step), so nothing crosses PCIe per step
(the reference samples on the CPU in 6 DataLoader
workers and copies every batch host->device, trainer.py:522-535).
"""
import ctypes

import numpy as np
import torch

from . import _lib as L
from .graph import csr_from_coo


class DeviceBPRSampler:
    def __init__(self, dataset, batch_size, device, seed=0, max_rounds=64):
        pairs = dataset.train_pairs if hasattr(dataset, 'train_pairs') else \
            np.asarray(dataset.train_array, np.int64).reshape(-1, 2)
        self.n_users, self.n_items = dataset.n_users, dataset.n_items
        # membership lists are sets: each user's distinct items, ascending - the duplicate-merging
        # CSR of the pairs (the multithreaded C++ builder; a numpy lexsort takes 20x as long)
        row_ptr, items, _, _ = csr_from_coo(pairs[:, 0], pairs[:, 1], self.n_users, self.n_items, None,
                                            dedup=True, want_eid=False)
        active = np.nonzero(np.diff(row_ptr) > 0)[0].astype(np.int32)
        if len(active) == 0:
            raise ValueError('no user has training items')
        self.device = torch.device(device)
        self.row_ptr = torch.from_numpy(row_ptr).to(self.device)
        self.items = torch.from_numpy(np.ascontiguousarray(items, dtype=np.int32)).to(self.device)
        self.active = torch.from_numpy(active).to(self.device)
        self.batch_size, self.seed, self.max_rounds = batch_size, int(seed), max_rounds
        self.length = len(dataset)
        self.step = 0

    def __len__(self):
        return (self.length + self.batch_size - 1) // self.batch_size

    def sample(self, n, offset=None, offset_dev=None):
        """One batch drawn at counter offset (default: this sampler's step count);
        with offset_dev (a device int64) the kernel adds *offset_dev on the device,
        so a captured hipGraph draws a new batch on every replay."""
        offset = self.step if offset is None else offset
        self.step += 1
        users = torch.empty(n, dtype=torch.int64, device=self.device)
        pos, neg = torch.empty_like(users), torch.empty_like(users)
        L.call('igr_bpr_sample', n, len(self.active), ctypes.c_void_p(self.active.data_ptr()),
               ctypes.c_void_p(self.row_ptr.data_ptr()), ctypes.c_void_p(self.items.data_ptr()), self.n_items,
               ctypes.c_uint64(self.seed), ctypes.c_uint64(offset),
               ctypes.c_void_p(0 if offset_dev is None else offset_dev.data_ptr()), self.max_rounds,
               ctypes.c_void_p(users.data_ptr()), ctypes.c_void_p(pos.data_ptr()), ctypes.c_void_p(neg.data_ptr()),
               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        return users, pos, neg

    def __iter__(self):
        left = self.length
        while left > 0:
            n = min(self.batch_size, left)
            left -= n
            yield self.sample(n)
