"""igr.config - the in-scope rows of the reference's config tables.

Same (dataset_config, model_config, trainer_config) dict triples as
config.py:1-527, restricted to the models of the hot path:
LightGCN / IGCN / IMF / NGCF on ML-1M (config.py:400-470) and Gowalla
(config.py:1-40), plus the synthetic benchmark graphs of BASELINE.json.
"""

TOPKS = [1, 5, 10, 15, 20, 25, 30, 35, 40, 45, 50, 55, 60, 65, 70, 75, 80, 85, 90, 95, 100]


def _trainer(name, lr, l2_reg, device, **kw):
    cfg = {'name': name, 'optimizer': 'Adam', 'lr': lr, 'l2_reg': l2_reg, 'device': device, 'n_epochs': 1000,
           'batch_size': 2048, 'dataloader_num_workers': 6, 'test_batch_size': 512, 'topks': TOPKS}
    cfg.update(kw)
    return cfg


def _rows(dataset_config, device):
    return [
        (dataset_config, {'name': 'LightGCN', 'embedding_size': 64, 'n_layers': 3, 'device': device},
         _trainer('BPRTrainer', 1.e-3, 1.e-4, device)),
        (dataset_config, {'name': 'IGCN', 'embedding_size': 64, 'n_layers': 3, 'device': device, 'dropout': 0.3,
                          'feature_ratio': 1.},
         _trainer('IGCNTrainer', 1.e-3, 0., device, aux_reg=0.01)),
        (dataset_config, {'name': 'NGCF', 'embedding_size': 64, 'layer_sizes': [64, 64, 64], 'device': device,
                          'dropout': 0.1},
         _trainer('BPRTrainer', 1.e-3, 1.e-3, device)),
        (dataset_config, {'name': 'IMF', 'embedding_size': 64, 'n_layers': 0, 'device': device, 'dropout': 0.1,
                          'feature_ratio': 1.},
         _trainer('IGCNTrainer', 1.e-3, 1.e-5, device, aux_reg=0.1)),
    ]


def get_ml_config(device, path='data/ml-1m/time'):
    """config.py:400-470 (ML-1M rows on the path)."""
    return _rows({'name': 'ProcessedDataset', 'path': path, 'device': device}, device)


def get_gowalla_config(device, path='data/Gowalla/time'):
    """config.py:1-40 (Gowalla rows on the path)."""
    return _rows({'name': 'ProcessedDataset', 'path': path, 'device': device}, device)


def get_synthetic_config(device, n_users=10_000_000, n_items=1_000_000, n_edges=200_000_000, d=64, seed=0,
                         item_dist='uniform'):
    """BASELINE.json configs[4] / north_star: synthetic bipartite graph."""
    ds = {'name': 'SyntheticDataset', 'n_users': n_users, 'n_items': n_items, 'n_edges': n_edges, 'seed': seed,
          'item_dist': item_dist, 'device': device}
    return [(ds, {'name': 'LightGCN', 'embedding_size': d, 'n_layers': 3, 'device': device},
             _trainer('BPRTrainer', 1.e-3, 1.e-4, device)),
            (ds, {'name': 'IGCN', 'embedding_size': d, 'n_layers': 3, 'device': device, 'dropout': 0.3,
                  'feature_ratio': 1.},
             _trainer('IGCNTrainer', 1.e-3, 0., device, aux_reg=0.01))]
