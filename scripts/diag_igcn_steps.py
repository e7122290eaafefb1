"""Diagnostic: per-step relative loss difference of igr's IGCN training against
the reference's first 20 step losses (tests/golden/train_<shape>.npz), to tell
fp32 noise (~1e-7) from a systematic difference."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
import ml_like  # noqa: E402
from igr import model as M  # noqa: E402
from igr import trainer as T  # noqa: E402


class DS:
    def __init__(self, name, n_users, n_items, train, val, test):
        self.name, self.n_users, self.n_items, self.device = name, n_users, n_items, 'cpu'
        self.train_data, self.val_data, self.test_data = train, val, test
        self.train_array = [[u, i] for u in range(n_users) for i in train[u]]
        self.train_pairs = np.array(self.train_array, dtype=np.int64)

    def __len__(self):
        return len(self.train_array)


def main(shape='ml100k', aux_reg=0.01, dropout=0.3):
    ref = np.load(os.path.join(ROOT, 'tests', 'golden', f'train_{shape}.npz'))
    nu, ni, mean_deg, d, L, epochs = ml_like.SHAPES[shape]
    train, val, test = ml_like.make_splits(nu, ni, mean_deg, seed=100)
    ds = DS(shape, nu, ni, train, val, test)
    bs = 2048
    spe = ml_like.steps_per_epoch(train, bs)
    main_b = ml_like.batches(train, ni, bs, spe, seed=1)
    aux_b = ml_like.batches(train, ni, bs, spe, seed=2)
    torch.manual_seed(int(ref['seed']))
    dev = torch.device('cuda')
    m = M.IGCN({'name': 'IGCN', 'embedding_size': d, 'n_layers': L, 'device': dev, 'dropout': dropout,
                'feature_ratio': 1., 'dataset': ds, 'dropout_rng': 'cpu'})
    tr = T.get_trainer({'name': 'IGCNTrainer', 'optimizer': 'Adam', 'lr': 1e-3, 'l2_reg': 0., 'aux_reg': aux_reg,
                        'device': dev, 'n_epochs': 1, 'batch_size': bs, 'test_batch_size': 512, 'topks': [20]},
                       ds, m)
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    m.train()
    for s in range(20):
        u, p, n = main_b[s]
        au, ap, an = aux_b[s]
        loss = tr.step(t(u), t(p), t(n), t(au), t(ap), t(an)).item()
        r = ref['first_step_losses'][s]
        print(f'step {s:2d} igr {loss:.8f} ref {r:.8f} rel {(loss - r) / r:+.2e}')


if __name__ == '__main__':
    main(*sys.argv[1:2])
