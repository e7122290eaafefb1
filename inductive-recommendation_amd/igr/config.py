"""igr.config - the reference's config tables (config.py:1-527) for the models of
the hot path.

`get_{gowalla,yelp,amazon,alibaba,ml}_config(device)` return, as there, a list of
(dataset_config, model_config, trainer_config) triples with the reference's
hyper-parameters, and every row sits at the reference's index (scripts pick a
row by position: [1] LightGCN, [2] IGCN, [4] NGCF, [6] IMF, [7] IMCGAE).  Rows whose
model lies outside this library (MF, ItemKNN, MultiVAE, IDCF, NeuMF, DOSE) are None.  `get_synthetic_config` adds the synthetic benchmark graphs.
"""

TOPKS = [1, 5, 10, 15, 20, 25, 30, 35, 40, 45, 50, 55, 60, 65, 70, 75, 80, 85, 90, 95, 100]


def _trainer(name, lr, l2_reg, device, **kw):
    cfg = {'name': name, 'optimizer': 'Adam', 'lr': lr, 'l2_reg': l2_reg, 'device': device, 'n_epochs': 1000,
           'batch_size': 2048, 'dataloader_num_workers': 6, 'test_batch_size': 512, 'topks': list(TOPKS)}
    cfg.update(kw)
    return cfg


def _table(path, device, n_rows, lgcn_l2=1.e-4, igcn_dropout=0.3, ngcf_dropout=0.1, ngcf_l2=1.e-3, imf_dropout=0.1,
           imcgae_dropout=0.3):
    """One dataset's table: the on-path rows at the reference's indices, None elsewhere."""
    ds = {'name': 'ProcessedDataset', 'path': path, 'device': device}
    rows = [None] * n_rows
    rows[1] = (ds, {'name': 'LightGCN', 'embedding_size': 64, 'n_layers': 3, 'device': device},
               _trainer('BPRTrainer', 1.e-3, lgcn_l2, device))
    rows[2] = (ds, {'name': 'IGCN', 'embedding_size': 64, 'n_layers': 3, 'device': device, 'dropout': igcn_dropout,
                    'feature_ratio': 1},
               _trainer('IGCNTrainer', 1.e-3, 0., device, aux_reg=0.01))
    rows[4] = (ds, {'name': 'NGCF', 'embedding_size': 64, 'layer_sizes': [64, 64, 64], 'device': device,
                    'dropout': ngcf_dropout},
               _trainer('BPRTrainer', 1.e-3, ngcf_l2, device))
    if imf_dropout is not None:
        rows[6] = (ds, {'name': 'IMF', 'embedding_size': 64, 'n_layers': 0, 'device': device, 'dropout': imf_dropout,
                        'feature_ratio': 1.},
                   _trainer('IGCNTrainer', 1.e-3, 1.e-5, device, aux_reg=0.1))
    rows[7] = (ds, {'name': 'IMCGAE', 'embedding_size': 64, 'n_layers': 3, 'device': device,
                    'dropout': imcgae_dropout},
               _trainer('BPRTrainer', 1.e-3, 0., device))
    return rows


def get_gowalla_config(device):
    """config.py:1-101."""
    return _table('data/Gowalla/time', device, 13)


def get_yelp_config(device):
    """config.py:103-204 (no IMF row: index 6 is a DOSE model there)."""
    return _table('data/Yelp/time', device, 13, ngcf_dropout=0.3, imf_dropout=None)


def get_amazon_config(device):
    """config.py:206-290."""
    return _table('data/Amazon/time', device, 11, lgcn_l2=1.e-5, igcn_dropout=0., ngcf_dropout=0.3, ngcf_l2=1.e-4,
                  imf_dropout=0.3, imcgae_dropout=0.9)


def get_alibaba_config(device):
    """config.py:292-409."""
    return _table('data/alibaba/time', device, 13)


def get_ml_config(device):
    """config.py:411-527."""
    return _table('data/ml-1m/time', device, 13)


def on_path(rows):
    """The rows of a table this library runs (the non-None ones)."""
    return [r for r in rows if r is not None]


def get_synthetic_config(device, n_users=10_000_000, n_items=1_000_000, n_edges=200_000_000, d=64, seed=0,
                         item_dist='uniform'):
    """The synthetic bipartite benchmark graph (10 M users x 1 M items x 200 M draws by default)."""
    ds = {'name': 'SyntheticDataset', 'n_users': n_users, 'n_items': n_items, 'n_edges': n_edges, 'seed': seed,
          'item_dist': item_dist, 'device': device}
    return [(ds, {'name': 'LightGCN', 'embedding_size': d, 'n_layers': 3, 'device': device},
             _trainer('BPRTrainer', 1.e-3, 1.e-4, device)),
            (ds, {'name': 'IGCN', 'embedding_size': d, 'n_layers': 3, 'device': device, 'dropout': 0.3,
                  'feature_ratio': 1.},
             _trainer('IGCNTrainer', 1.e-3, 0., device, aux_reg=0.01))]
