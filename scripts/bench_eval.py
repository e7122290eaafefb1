"""Where one eval (trainer.py:146-210) spends its time at the ML-1M shape: the ranking on the
GPU (one propagation, score GEMM, mask, top-k, one copy) and the metrics on the host."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import ml_like
    from igr import model as M
    from igr import trainer as T
    shape = sys.argv[1] if len(sys.argv) > 1 else 'ml1m_l3'
    nu, ni, mean_deg, d, L, _ = ml_like.SHAPES[shape]
    train, val, test = ml_like.make_splits(nu, ni, mean_deg, seed=100)

    class DS:
        name, n_users, n_items = shape, nu, ni
        train_data, val_data, test_data = train, val, test
        train_array = [[u, i] for u in range(nu) for i in train[u]]
        train_pairs = np.array(train_array, dtype=np.int64)

        def __len__(self):
            return len(self.train_array)
    dev = torch.device('cuda')
    m = M.IGCN({'name': 'IGCN', 'embedding_size': d, 'n_layers': L, 'device': dev, 'dropout': 0.3, 'feature_ratio': 1.,
                'dataset': DS()})
    out = {'shape': shape}
    for static in (False, True):
        tr = T.BasicTrainer({'name': 'BasicTrainer', 'dataset': DS(), 'model': m, 'topks': [1, 5, 10, 15, 20],
                             'device': dev, 'n_epochs': 0, 'test_batch_size': 512, 'static_eval_lists': static})
        for _ in range(3):
            tr.eval('test')
        torch.cuda.synchronize()
        t = {'rank': 0., 'metrics': 0.}
        n = 20
        for _ in range(n):
            t0 = time.perf_counter()
            rec = tr.rank('test')
            t1 = time.perf_counter()
            tr.calculate_metrics(tr.dataset.test_data, rec)
            t2 = time.perf_counter()
            t['rank'] += (t1 - t0) / n
            t['metrics'] += (t2 - t1) / n
        out['static_lists' if static else 'lists_read_every_eval'] = {k: round(v * 1e3, 3) for k, v in t.items()}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
