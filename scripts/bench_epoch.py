"""End-to-end epochs at the ML-1M shape: the reference's training loop body
(IGCNTrainer.train_one_epoch + eval on val and test, trainer.py:58-113 /
518-561) on MovieLens-shaped synthetic data (tests/golden/ml_like.py, the same
data the training-parity test uses), timed per epoch, eager and with the
hipGraph-captured step.  The reference's own CPU time per epoch on this data is
in tests/golden/train_ml1m*.npz's generator log (make_train_golden.py prints it)."""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument('--shape', default='ml1m_l3')
    ap.add_argument('--epochs', type=int, default=10)
    args = ap.parse_args()
    import ml_like
    from igr import model as M
    from igr import trainer as T
    nu, ni, mean_deg, d, L, _ = ml_like.SHAPES[args.shape]
    train, val, test = ml_like.make_splits(nu, ni, mean_deg, seed=100)

    class DS:
        name, n_users, n_items = args.shape, nu, ni
        train_data, val_data, test_data = train, val, test
        train_array = [[u, i] for u in range(nu) for i in train[u]]
        train_pairs = np.array(train_array, dtype=np.int64)

        def __len__(self):
            return len(self.train_array)
    dev = torch.device('cuda')
    out = {'shape': args.shape, 'n_users': nu, 'n_items': ni, 'train_interactions': len(DS.train_array), 'd': d,
           'layers': L}
    for graph in (False, True):
        torch.manual_seed(7)
        m = M.IGCN({'name': 'IGCN', 'embedding_size': d, 'n_layers': L, 'device': dev, 'dropout': 0.3,
                    'feature_ratio': 1., 'dataset': DS()})
        tr = T.get_trainer({'name': 'IGCNTrainer', 'optimizer': 'Adam', 'lr': 1e-3, 'l2_reg': 0., 'aux_reg': 0.01,
                            'device': dev, 'n_epochs': args.epochs, 'batch_size': 2048, 'test_batch_size': 512,
                            'topks': [1, 5, 10, 15, 20], 'graph': graph, 'seed': 1,
                            'static_eval_lists': True}, DS(), m)  # as inside train(): the lists stay put
        ep_s, recall, parts = [], [], []
        for _ in range(args.epochs):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.train()
            tr.train_one_epoch()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            _, vm, _ = tr.eval('val')
            t2 = time.perf_counter()
            _, tm, _ = tr.eval('test')
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            ep_s.append(t3 - t0)
            parts.append((t1 - t0, t2 - t1, t3 - t2))
            recall.append(float(tm['Recall'][20]))
        key = 'graph' if graph else 'eager'
        med = np.median(np.array(parts[1:]), axis=0)
        out[key] = {'epoch_s_first': ep_s[0], 'epoch_s_median_rest': float(np.median(ep_s[1:])),
                    'train_s': float(med[0]), 'eval_val_s': float(med[1]), 'eval_test_s': float(med[2]),
                    'test_recall20_per_epoch': recall}
        print(key, out[key], file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
