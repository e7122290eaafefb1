"""Generate tests/golden/imcgae.npz by RUNNING the reference's IMCGAE (model.py:4300-4345)
on the 'uni' and 'pow' graphs of make_golden.py: representation and embedding gradient in
eval mode, and the train-mode representation with the node-dropout masks drawn from the CPU
generator at a fixed seed.  Same stubs as make_golden.py.

Run:  python tests/golden/make_imcgae_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G  # noqa: E402

D, L, DROPOUT, TRAIN_SEED = 32, 3, 0.3, 41


def main():
    torch.set_num_threads(4)
    fx = {'d': np.int64(D), 'n_layers': np.int64(L), 'dropout': np.float64(DROPOUT), 'train_seed': np.int64(TRAIN_SEED)}
    for cname in ['uni', 'pow']:
        nu, ni, spec = G.CASES[cname]
        edges = G.make_edges(spec[0], nu, ni, spec[1], spec[2])
        ds = G.ToyDataset(nu, ni, edges, name=cname)
        torch.manual_seed(700)
        m = G.ref_model.IMCGAE({'name': 'IMCGAE', 'embedding_size': D, 'n_layers': L, 'device': 'cpu',
                                'dropout': DROPOUT, 'dataset': ds})
        m.eval()
        fx[cname + '_emb'] = m.embedding.weight.detach().numpy().copy()
        rep = m.get_rep()
        fx[cname + '_rep'] = rep.detach().numpy().copy()
        R = torch.randn(rep.shape, generator=torch.Generator().manual_seed(10))
        (rep * R).sum().backward()
        fx[cname + '_R'] = R.numpy()
        fx[cname + '_grad'] = m.embedding.weight.grad.numpy().copy()
        m.train()
        torch.manual_seed(TRAIN_SEED)
        with torch.no_grad():
            fx[cname + '_train_rep'] = m.get_rep().numpy().copy()
        m.eval()
        with torch.no_grad():
            users = torch.arange(0, nu, 37)
            fx[cname + '_predict_users'] = users.numpy()
            fx[cname + '_predict_scores'] = m.predict(users).numpy().copy()
    path = os.path.join(HERE, 'imcgae.npz')
    np.savez_compressed(path, **fx)
    print('wrote', path, os.path.getsize(path))


if __name__ == '__main__':
    main()
