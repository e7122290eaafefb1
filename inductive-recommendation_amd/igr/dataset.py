"""igr.dataset - the reference's dataset surface (dataset.py) for the path.

ProcessedDataset reads the same train/val/test.txt format
(dataset.py:140-164); BasicDataset.__getitem__ is the reference's BPR
sampler (dataset.py:119-131).  BPRBatchSampler draws whole batches with the
same distribution in vectorised numpy (the reference runs the per-sample
Python sampler in 6 DataLoader workers, trainer.py:522-526).
SyntheticDataset builds the benchmark's random bipartite graphs;
GowallaDataset / YelpDataset / AmazonDataset / MovieLensDataset ingest raw logs.
"""
import os
import random
import sys

import numpy as np


def get_dataset(config):
    """dataset.py:10-14."""
    config = config.copy()
    dataset = getattr(sys.modules[__name__], config['name'])
    return dataset(config)


class BasicDataset:
    """dataset.py:47-137 (attributes and sampler)."""

    def __init__(self, dataset_config):
        self.config = dataset_config
        self.name = dataset_config['name']
        self.device = dataset_config.get('device', 'cpu')
        self.negative_sample_ratio = dataset_config.get('neg_ratio', 1)
        self.n_users = 0
        self.n_items = 0
        self.train_data = None
        self.val_data = None
        self.test_data = None
        self.train_array = None
        self._pairs = None

    @property
    def train_pairs(self):
        """train_array as int64 [E, 2] (cached)."""
        if self._pairs is None:
            self._pairs = np.asarray(self.train_array, dtype=np.int64).reshape(-1, 2)
        return self._pairs

    def __len__(self):
        return len(self.train_array)

    def __getitem__(self, index):
        """dataset.py:119-131 verbatim semantics: uniform user with training
        items, uniform positive, rejection-sampled negative."""
        user = random.randint(0, self.n_users - 1)
        while not self.train_data[user]:
            user = random.randint(0, self.n_users - 1)
        pos_item = np.random.choice(self.train_data[user])
        data = [[user, pos_item] for _ in range(self.negative_sample_ratio)]
        for idx in range(self.negative_sample_ratio):
            neg_item = random.randint(0, self.n_items - 1)
            while neg_item in self.train_data[user]:
                neg_item = random.randint(0, self.n_items - 1)
            data[idx].append(neg_item)
        return np.array(data, dtype=np.int64)

    def output_dataset(self, path):
        """dataset.py:133-137."""
        os.makedirs(path, exist_ok=True)
        for name, data in [('train.txt', self.train_data), ('val.txt', self.val_data), ('test.txt', self.test_data)]:
            output_data(os.path.join(path, name), data)


def output_data(file_path, data):
    """dataset.py:40-44: one line per user, 'user item item ...'."""
    with open(file_path, 'w') as f:
        for user in range(len(data)):
            f.write(' '.join([str(user)] + [str(i) for i in data[user]]) + '\n')


def read_split(file_path):
    """dataset.py:156-164: one line per user, 'user item item ...'."""
    data, n_items = [], 0
    with open(file_path) as f:
        lines = f.read().strip().split('\n')
    for line in lines:
        items = [int(x) for x in line.split(' ')[1:]]
        if items:
            n_items = max(n_items, max(items) + 1)
        data.append(items)
    return data, n_items


def ingest(raw_users, raw_items, times, min_inter, split_ratio):
    """Vectorised restatement of the reference's raw pipeline:
      remove_sparse_ui (dataset.py:66-92): iterative k-core on unique (user, item)
        pairs - users with < min_inter items removed, then items with < min_inter
        users, repeated until stable; survivors numbered in first-appearance order;
      update_user_inter_lists (dataset.py:27-37): one entry per (user, item), the
        earliest time, listed in first-appearance order;
      generate_data (dataset.py:94-114): per-user stable sort by time, then
        train = [:int(n*r0)], val = [int(n*r0):-int(n*r2)], test = [-int(n*r2):]
        (with int(n*r2) == 0 the reference's slices give val = [] and test = the
        whole list; kept as is).
    Inputs are per-line arrays in file order; returns (train, val, test, n_users, n_items)."""
    raw_users, raw_items = np.asarray(raw_users), np.asarray(raw_items)
    times = np.asarray(times, np.int64)

    def first_order_codes(x):
        uniq, first, inv = np.unique(x, return_index=True, return_inverse=True)
        rank = np.empty(len(uniq), np.int64)
        rank[np.argsort(first, kind='stable')] = np.arange(len(uniq))
        return rank[inv], len(uniq)
    uc, nu0 = first_order_codes(raw_users)
    ic, ni0 = first_order_codes(raw_items)
    key = uc * ni0 + ic
    ukey, kfirst = np.unique(key, return_index=True)
    pu, pi = ukey // ni0, ukey % ni0
    alive_u, alive_i = np.ones(nu0, bool), np.ones(ni0, bool)
    live = np.ones(len(ukey), bool)
    while True:
        du = np.bincount(pu[live], minlength=nu0)
        drop_u = alive_u & (du < min_inter)
        alive_u &= ~drop_u
        live &= alive_u[pu]
        di = np.bincount(pi[live], minlength=ni0)
        drop_i = alive_i & (di < min_inter)
        alive_i &= ~drop_i
        live &= alive_i[pi]
        if not drop_u.any() and not drop_i.any():
            break
    umap = np.cumsum(alive_u) - 1
    imap = np.cumsum(alive_i) - 1
    n_users, n_items = int(alive_u.sum()), int(alive_i.sum())
    # earliest time per kept pair; order = (user, time, first appearance of the pair)
    pos = np.searchsorted(ukey, key)
    tmin = np.full(len(ukey), np.iinfo(np.int64).max, np.int64)
    np.minimum.at(tmin, pos, times)
    sel = np.nonzero(live)[0]
    order = np.lexsort((kfirst[sel], tmin[sel], umap[pu[sel]]))
    sel = sel[order]
    users, items = umap[pu[sel]], imap[pi[sel]]
    ptr = np.searchsorted(users, np.arange(n_users + 1))
    train, val, test = [], [], []
    for u in range(n_users):
        lst = items[ptr[u]:ptr[u + 1]].tolist()
        k = len(lst)
        n_tr, n_te = int(k * split_ratio[0]), int(k * split_ratio[2])
        train.append(lst[:n_tr])
        val.append(lst[n_tr:-n_te] if n_te else [])
        test.append(lst[-n_te:] if n_te else lst)
    return train, val, test, n_users, n_items


class InteractionDataset(BasicDataset):
    """Raw interaction logs -> train / val / test via `ingest` (the reference's
    GowallaDataset pipeline); train_array is filled (the reference leaves it
    empty and relies on ProcessedDataset re-reading the files it writes)."""

    def load(self, raw_users, raw_items, times):
        self.train_data, self.val_data, self.test_data, self.n_users, self.n_items = ingest(
            raw_users, raw_items, times, self.config['min_inter'], self.config['split_ratio'])
        self.train_array = [[u, i] for u in range(self.n_users) for i in self.train_data[u]]


class GowallaDataset(InteractionDataset):
    """dataset.py:167-189: Gowalla_totalCheckins.txt ('user<TAB>time<TAB>lat<TAB>lon<TAB>loc').
    Times are parsed as UTC (the reference uses time.mktime: local time; only the
    order matters, identical unless the host zone has DST jumps)."""

    def __init__(self, dataset_config):
        super().__init__(dataset_config)
        import pandas as pd
        df = pd.read_csv(os.path.join(dataset_config['path'], 'Gowalla_totalCheckins.txt'), sep='\t', header=None,
                         names=['u', 't', 'lat', 'lon', 'i'], dtype={'u': np.int64, 't': str, 'i': np.int64})
        # the file's '%Y-%m-%dT%H:%M:%SZ' stamps are ISO 8601: pandas' ISO parser reads them 3x faster
        # than its strptime path (1 M lines: 1.1 s against 3.3 s), to the same seconds
        t = pd.to_datetime(df['t'], format='ISO8601', utc=True).astype('int64') // 10 ** 9
        self.load(df['u'].to_numpy(), df['i'].to_numpy(), t.to_numpy())


def _first_appearance_codes(ids):
    """String ids -> int codes numbered in first-appearance order (what the
    reference's insertion-ordered dicts give), so `ingest` sees the same order."""
    import pandas as pd
    return pd.factorize(np.asarray(ids, dtype=object), sort=False)[0].astype(np.int64)


class YelpDataset(InteractionDataset):
    """dataset.py:192-223: yelp_academic_dataset_review.json (one JSON record per
    line); reviews with stars > 3 are interactions, time = 'date'
    ('%Y-%m-%d %H:%M:%S', parsed as UTC like GowallaDataset)."""

    def __init__(self, dataset_config):
        super().__init__(dataset_config)
        import pandas as pd
        path = os.path.join(dataset_config['path'], 'yelp_academic_dataset_review.json')
        us, its, ts = [], [], []
        for chunk in pd.read_json(path, lines=True, dtype=False, convert_dates=False, keep_default_dates=False,
                                  chunksize=1 << 20):
            keep = chunk['stars'].astype(np.float64).to_numpy() > 3.
            c = chunk[keep]
            us.append(c['user_id'].astype(str).to_numpy())
            its.append(c['business_id'].astype(str).to_numpy())
            ts.append((pd.to_datetime(c['date'], format='%Y-%m-%d %H:%M:%S', utc=True).astype('int64')
                       // 10 ** 9).to_numpy())
        cat = lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dt)  # noqa: E731
        self.load(_first_appearance_codes(cat(us, object)), _first_appearance_codes(cat(its, object)),
                  cat(ts, np.int64))


class AmazonDataset(InteractionDataset):
    """dataset.py:226-255: ratings_Books.csv ('user,item,rating,time', no header);
    ratings > 3 are interactions (the Amazon-Books config of BASELINE.json)."""

    def __init__(self, dataset_config):
        super().__init__(dataset_config)
        import pandas as pd
        df = pd.read_csv(os.path.join(dataset_config['path'], 'ratings_Books.csv'), header=None,
                         names=['u', 'i', 'r', 't'], dtype={'u': str, 'i': str, 'r': np.float64, 't': np.int64})
        df = df[df['r'].to_numpy() > 3.]
        self.load(_first_appearance_codes(df['u'].to_numpy()), _first_appearance_codes(df['i'].to_numpy()),
                  df['t'].to_numpy())


class MovieLensDataset(InteractionDataset):
    """MovieLens ratings (no loader exists in the reference): ML-1M/10M
    'ratings.dat' (user::movie::rating::time) or ML-100K 'u.data'
    (tab-separated).  Ratings >= config['min_rating'] (default: all) are
    interactions; the rest of the pipeline is the GowallaDataset one."""

    def __init__(self, dataset_config):
        super().__init__(dataset_config)
        import pandas as pd
        path = dataset_config['path']
        f_dat, f_tab = os.path.join(path, 'ratings.dat'), os.path.join(path, 'u.data')
        if os.path.exists(f_dat):
            raw = pd.read_csv(f_dat, sep='::', header=None, engine='python').to_numpy(np.int64)
        elif os.path.exists(f_tab):
            raw = pd.read_csv(f_tab, sep='\t', header=None).to_numpy(np.int64)
        else:
            raise FileNotFoundError(f'no ratings.dat or u.data under {path}')
        raw = raw[raw[:, 2] >= dataset_config.get('min_rating', -np.inf)]
        self.load(raw[:, 0], raw[:, 1], raw[:, 3])


class ProcessedDataset(BasicDataset):
    """dataset.py:140-164."""

    def __init__(self, dataset_config):
        super().__init__(dataset_config)
        path = dataset_config['path']
        self.train_data, a = read_split(os.path.join(path, 'train.txt'))
        self.val_data, b = read_split(os.path.join(path, 'val.txt'))
        self.test_data, c = read_split(os.path.join(path, 'test.txt'))
        self.n_items = max(a, b, c)
        assert len(self.train_data) == len(self.val_data) == len(self.test_data)
        self.n_users = len(self.train_data)
        self.train_array = [[u, i] for u in range(self.n_users) for i in self.train_data[u]]

    def read_data(self, file_path):
        """dataset.py:156-164, by its name there: the lists of one split file; n_items grows to cover them."""
        data, n = read_split(file_path)
        self.n_items = max(self.n_items, n)
        return data


class AuxiliaryDataset(BasicDataset):
    """dataset.py:258-273: the training data restricted to, and renumbered by, the
    template-feature maps of an inductive model (user u -> user_map[u], item i ->
    item_map[i]; pairs with an unmapped end are left out).  Vectorised over the
    pair array; the per-user lists (same order as the dataset's) are built only if
    a host-side sampler asks for them."""

    def __init__(self, dataset, user_map, item_map):
        self.name = 'AuxiliaryDataset'
        self.n_users = len(user_map)
        self.n_items = len(item_map)
        self.device = getattr(dataset, 'device', 'cpu')
        self.negative_sample_ratio = 1
        self.length = len(dataset)
        pairs = dataset.train_pairs if hasattr(dataset, 'train_pairs') else \
            np.asarray(dataset.train_array, dtype=np.int64).reshape(-1, 2)
        u = _map_array(user_map, dataset.n_users)[pairs[:, 0]]
        i = _map_array(item_map, dataset.n_items)[pairs[:, 1]]
        keep = (u >= 0) & (i >= 0)
        self._pairs = np.stack([u[keep], i[keep]], axis=1)  # in the dataset's pair order
        self.train_array = self._pairs
        self._train_data = None
        self.val_data = self.test_data = None

    @property
    def train_data(self):
        if self._train_data is None:
            # train_array lists each user's items in train_data order (dataset.py:155-160), so a
            # stable sort by the new user id gives the reference's lists
            order = np.argsort(self._pairs[:, 0], kind='stable')
            ptr = np.searchsorted(self._pairs[order, 0], np.arange(self.n_users + 1))
            items = self._pairs[order, 1]
            self._train_data = _lists(items, ptr)
        return self._train_data

    @train_data.setter
    def train_data(self, v):
        self._train_data = v

    def __len__(self):
        return self.length


def _lists(items, ptr):
    """CSR (items, row_ptr) as a list of per-row Python lists (one tolist, then slices)."""
    flat, p = items.tolist(), ptr.tolist()
    return [flat[a:b] for a, b in zip(p[:-1], p[1:])]


def _map_array(id_map, n):
    """A {old id: new id} dict as an int64 lookup array over [0, n), -1 where unmapped."""
    a = np.full(n, -1, np.int64)
    if id_map:
        a[np.fromiter(id_map.keys(), np.int64, len(id_map))] = np.fromiter(id_map.values(), np.int64, len(id_map))
    return a


class SyntheticDataset(BasicDataset):
    """Random bipartite interactions: users ~ U[0, n_users),
    items ~ U[0, n_items) or Zipf(s) ; duplicates kept in train_array and
    summed by the graph build exactly as utils.generate_daj_mat does.
    val/test hold `n_eval` random items per user (synthetic; metrics are not
    meaningful, only shapes)."""

    def __init__(self, dataset_config):
        super().__init__(dataset_config)
        self.n_users = int(dataset_config['n_users'])
        self.n_items = int(dataset_config['n_items'])
        n_edges = int(dataset_config['n_edges'])
        seed = int(dataset_config.get('seed', 0))
        self._pairs = synthetic_pairs(self.n_users, self.n_items, n_edges, seed,
                                      dataset_config.get('item_dist', 'uniform'), dataset_config.get('zipf_s', 1.1))
        self.train_array = self._pairs
        self._train_data = None
        self.val_data = self.test_data = None

    @property
    def train_data(self):
        if self._train_data is None and self._pairs is not None:
            order = np.argsort(self._pairs[:, 0], kind='stable')
            items = self._pairs[order, 1]
            ptr = np.searchsorted(self._pairs[order, 0], np.arange(self.n_users + 1))
            self._train_data = _lists(items, ptr)
        return self._train_data

    @train_data.setter
    def train_data(self, v):
        self._train_data = v


def synthetic_pairs(n_users, n_items, n_edges, seed=0, item_dist='uniform', zipf_s=1.1, stacked=True):
    """int64 [n_edges, 2] (user, item) draws with torch's CPU generator; stacked=False
    returns the two int64 arrays (users, items) of the same draws instead."""
    import torch
    g = torch.Generator().manual_seed(seed)
    u = torch.randint(0, n_users, (n_edges,), generator=g, dtype=torch.int64)
    if item_dist == 'uniform':
        i = torch.randint(0, n_items, (n_edges,), generator=g, dtype=torch.int64)
    elif item_dist == 'zipf':
        w = 1.0 / torch.arange(1, n_items + 1, dtype=torch.float64) ** zipf_s
        i = torch.multinomial(w / w.sum(), n_edges, replacement=True, generator=g)
    else:
        raise ValueError(item_dist)
    if not stacked:
        return u.numpy(), i.numpy()
    return torch.stack([u, i], 1).numpy()


class BPRBatchSampler:
    """Vectorised BasicDataset.__getitem__ (dataset.py:119-131): a batch of
    (user, pos, neg) with user uniform over users that have training items,
    pos uniform over the user's items, neg uniform over items the user has
    not interacted with (rejection)."""

    def __init__(self, dataset, batch_size, seed=None):
        pairs = dataset.train_pairs if hasattr(dataset, 'train_pairs') else \
            np.asarray(dataset.train_array, np.int64).reshape(-1, 2)
        self.n_users, self.n_items = dataset.n_users, dataset.n_items
        self.batch_size = batch_size
        self.length = len(dataset)
        order = np.lexsort((pairs[:, 1], pairs[:, 0]))
        p = pairs[order]
        self.items = p[:, 1].copy()
        self.ptr = np.searchsorted(p[:, 0], np.arange(self.n_users + 1))
        self.deg = np.diff(self.ptr)
        self.active = np.nonzero(self.deg > 0)[0]
        self.keys = np.unique(p[:, 0] * self.n_items + p[:, 1])
        self.rng = np.random.default_rng(seed)

    def __len__(self):
        return (self.length + self.batch_size - 1) // self.batch_size

    def sample(self, n):
        users = self.active[self.rng.integers(0, len(self.active), n)]
        pos = self.items[self.ptr[users] + (self.rng.random(n) * self.deg[users]).astype(np.int64)]
        neg = self.rng.integers(0, self.n_items, n)
        bad = self._member(users, neg)
        while bad.any():
            neg[bad] = self.rng.integers(0, self.n_items, int(bad.sum()))
            bad[bad] = self._member(users[bad], neg[bad])
        return users, pos, neg

    def _member(self, users, items):
        k = users * self.n_items + items
        j = np.searchsorted(self.keys, k)
        j = np.minimum(j, len(self.keys) - 1)
        return self.keys[j] == k

    def __iter__(self):
        left = self.length
        while left > 0:
            n = min(self.batch_size, left)
            left -= n
            yield self.sample(n)
