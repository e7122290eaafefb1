"""igr.utils - utils.py helpers the trainers use (utils.py:13-30, 280-305)."""
import os
import random
import sys

import numpy as np
import torch


def set_seed(seed=0):
    """utils.py:13-21."""
    random.seed(seed)
    os.environ['PYTHONHASHSEED'] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


class Unbuffered:
    """utils.py:291-305."""

    def __init__(self, stream):
        self.stream = stream

    def write(self, data):
        self.stream.write(data)
        self.stream.flush()

    def writelines(self, datas):
        self.stream.writelines(datas)
        self.stream.flush()

    def __getattr__(self, attr):
        return getattr(self.stream, attr)


def init_run(log_path, seed):
    """utils.py:24-30: seed, then redirect stdout/stderr to log_path/lo00gg.txt."""
    set_seed(seed)
    os.makedirs(log_path, exist_ok=True)
    f = Unbuffered(open(os.path.join(log_path, 'lo00gg.txt'), 'w'))
    sys.stderr = f
    sys.stdout = f


class AverageMeter:
    """utils.py:280-288."""

    def __init__(self):
        self.avg = 0.
        self.sum = 0.
        self.count = 0.

    def update(self, val, n=1):
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count
