"""igr.utils - run set-up helpers with the names the reference's scripts call
(`set_seed`, `init_run`; /root/reference utils.py:13-30).  The epoch loss is
accumulated on the device by the trainers, so no host-side meter is needed."""
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
