"""Deterministic MovieLens-shaped interaction data and BPR batches (pure numpy).

Shared by tests/golden/make_train_golden.py (which trains the REFERENCE on it)
and tests/test_gpu_training_parity.py (which trains igr on it): both sides
see the same splits and the same (user, pos, neg) batches, so their
trajectories can be compared step for step.

The data is synthetic (no MovieLens files exist in the reference or the
image): a rank-8 preference model with Zipf item popularity, per-user
lognormal activity (>= 20 interactions, as ML's 20-rating minimum), then a
per-user 80/10/10 split in (synthetic) time order - the shape of
BasicDataset.generate_data (dataset.py:94-114) with split_ratio [0.8, 0.1, 0.1].
"""
import numpy as np

SHAPES = {
    # name: (n_users, n_items, mean interactions per user, d, n_layers, epochs)
    'ml100k': (943, 1682, 106, 32, 1, 20),
    'ml1m': (6040, 3706, 165, 64, 2, 10),
    # the reference's own IGCN depth (config.py:430: n_layers 3, d 64) on the ML-1M shape
    'ml1m_l3': (6040, 3706, 165, 64, 3, 10),
}


# The Gowalla shape of BASELINE's third configuration (29,858 users x 40,981 items,
# ~1.03 M training interactions, d = 128, 3 layers; /root/reference config.py:12-23):
# (n_users, n_items, mean interactions per user, d, n_layers, epochs)
SHAPES['gowalla'] = (29858, 40981, 43, 128, 3, 2)


def zipf_splits(n_users, n_items, mean_deg, seed, min_deg=10):
    """Vectorised synthetic interactions for shapes too large for make_splits'
    dense preference matrix: per-user lognormal activity (>= min_deg, Gowalla's
    10-core), items drawn from a Zipf(0.9) popularity law (repeats dropped), a
    random interaction-time order per user and the same per-user 80/10/10 split
    (dataset.py:94-114).  Returns (train, val, test) lists of sorted item lists."""
    rng = np.random.default_rng(seed)
    deg = np.clip(rng.lognormal(np.log(mean_deg) - 0.3, 0.8, n_users), min_deg, n_items // 4).astype(np.int64)
    w = 1.0 / np.arange(1, n_items + 1) ** 0.9
    perm = rng.permutation(n_items)
    # draw 30 % extra so that most users still reach their degree after repeats are dropped
    draws = (deg * 1.3).astype(np.int64) + 2
    u = np.repeat(np.arange(n_users, dtype=np.int64), draws)
    i = perm[rng.choice(n_items, size=int(draws.sum()), p=w / w.sum())]
    key = np.unique(u * n_items + i)
    u, i = key // n_items, key % n_items
    t = rng.random(len(u))  # synthetic interaction time
    order = np.lexsort((t, u))
    u, i = u[order], i[order]
    ptr = np.searchsorted(u, np.arange(n_users + 1))
    train, val, test = [], [], []
    for x in range(n_users):
        items = i[ptr[x]:ptr[x + 1]][:deg[x]]
        n_tr, n_te = int(len(items) * 0.8), int(len(items) * 0.1)
        train.append(sorted(items[:n_tr].tolist()))
        val.append(sorted(items[n_tr:len(items) - n_te].tolist()))
        test.append(sorted(items[len(items) - n_te:].tolist()))
    return train, val, test


def batches_vec(train_data, n_items, batch_size, n_steps, seed):
    """batches() for large shapes, vectorised: the same distribution (user uniform
    over users with training items, positive uniform over the user's items,
    negative uniform over the items the user has not interacted with, by
    rejection; dataset.py:119-131)."""
    rng = np.random.default_rng(seed)
    lens = np.array([len(x) for x in train_data], np.int64)
    ptr = np.concatenate([[0], np.cumsum(lens)])
    flat = np.fromiter((i for x in train_data for i in x), np.int64, count=int(ptr[-1]))
    users_ok = np.nonzero(lens > 0)[0].astype(np.int64)
    keys = np.repeat(np.arange(len(train_data), dtype=np.int64), lens) * n_items + flat  # sorted
    out = []
    for _ in range(n_steps):
        u = users_ok[rng.integers(0, len(users_ok), batch_size)]
        p = flat[ptr[u] + (rng.random(batch_size) * lens[u]).astype(np.int64)]
        n = rng.integers(0, n_items, batch_size)
        while True:
            k = u * n_items + n
            j = np.minimum(np.searchsorted(keys, k), len(keys) - 1)
            bad = np.nonzero(keys[j] == k)[0]
            if len(bad) == 0:
                break
            n[bad] = rng.integers(0, n_items, len(bad))
        out.append((u, p, n))
    return out


def splits_for(shape, seed=100):
    """The (train, val, test) lists of a named shape."""
    nu, ni, mean_deg = SHAPES[shape][:3]
    return zipf_splits(nu, ni, mean_deg, seed) if shape == 'gowalla' else make_splits(nu, ni, mean_deg, seed)


def batches_for(shape, train_data, n_items, batch_size, n_steps, seed):
    fn = batches_vec if shape == 'gowalla' else batches
    return fn(train_data, n_items, batch_size, n_steps, seed)


def _name_seed(name):
    import zlib
    return zlib.crc32(name.encode()) & 0x7fffffff


def scale_params(name, n_rows, d, heads=0):
    """Model parameters of a BASELINE-sized fixture (tests/golden/make_scale_golden.py):
    numpy legacy streams, identical wherever they are drawn.  emb ~ N(0, 0.1^2)
    (model.py:4124); with heads, the d -> heads * d projections of AttIGCN drawn
    as nn.Linear draws them, U(-1/sqrt(d), 1/sqrt(d))."""
    rs = np.random.RandomState(_name_seed(name))
    P = {'emb': (rs.standard_normal((n_rows, d)) * 0.1).astype(np.float32)}
    if heads:
        b = 1.0 / np.sqrt(d)
        for k, shp in [('wq', (heads * d, d)), ('bq', (heads * d,)), ('wk', (heads * d, d)), ('bk', (heads * d,))]:
            P[k] = rs.uniform(-b, b, shp).astype(np.float32)
    return P


def scale_samples(name, n_nodes, nnz_feat, nnz_adj=None):
    """The rows / edges whose values a BASELINE-sized fixture keeps: 512 node rows,
    512 rows of the feature table (its last two, the general features every node
    reads, always among them), 4096 edges of the feature graph (and of the
    adjacency)."""
    rs = np.random.RandomState(_name_seed(name) ^ 0x5bd1e995)
    rows = np.unique(np.concatenate([[0, n_nodes - 1], rs.randint(0, n_nodes, 510)]))
    feat_rows = np.unique(np.concatenate([[0, n_nodes, n_nodes + 1], rs.randint(0, n_nodes + 2, 509)]))
    out = {'rows': rows, 'feat_rows': feat_rows, 'edges': np.unique(rs.randint(0, nnz_feat, 4096))}
    if nnz_adj is not None:
        out['adj_edges'] = np.unique(rs.randint(0, nnz_adj, 4096))
    return out


def scale_cotangent(shape):
    """The fixed cotangent R of the gradient fixtures: gradients of sum(rep * R)."""
    return np.random.RandomState(8).standard_normal(shape).astype(np.float32)


def make_splits(n_users, n_items, mean_deg, seed):
    rng = np.random.default_rng(seed)
    P = rng.normal(size=(n_users, 8))
    Q = rng.normal(size=(n_items, 8))
    pop = np.log(1.0 / np.arange(1, n_items + 1) ** 0.9)
    rng.shuffle(pop)
    logits = P @ Q.T / 2.0 + pop[None, :]
    deg = np.clip(rng.lognormal(np.log(mean_deg) - 0.3, 0.8, n_users), 20, n_items // 2).astype(np.int64)
    train, val, test = [], [], []
    for u in range(n_users):
        g = rng.gumbel(size=n_items)
        items = np.argsort(-(logits[u] + g))[:deg[u]]
        items = items[rng.permutation(len(items))]  # synthetic interaction time order
        n_tr, n_te = int(len(items) * 0.8), int(len(items) * 0.1)
        train.append(sorted(items[:n_tr].tolist()))
        val.append(sorted(items[n_tr:len(items) - n_te].tolist()))
        test.append(sorted(items[len(items) - n_te:].tolist()))
    return train, val, test


def batches(train_data, n_items, batch_size, n_steps, seed):
    """n_steps batches of (users, pos, neg) with the distribution of
    BasicDataset.__getitem__ (dataset.py:119-131)."""
    rng = np.random.default_rng(seed)
    users_ok = np.array([u for u in range(len(train_data)) if train_data[u]], np.int64)
    sets = [set(x) for x in train_data]
    out = []
    for _ in range(n_steps):
        u = users_ok[rng.integers(0, len(users_ok), batch_size)]
        p = np.array([train_data[x][rng.integers(0, len(train_data[x]))] for x in u], np.int64)
        n = rng.integers(0, n_items, batch_size)
        for k in range(batch_size):
            while n[k] in sets[u[k]]:
                n[k] = rng.integers(0, n_items)
        out.append((u, p, n))
    return out


def steps_per_epoch(train_data, batch_size):
    n = sum(len(x) for x in train_data)
    return (n + batch_size - 1) // batch_size


def write_checkins(path, n_users=300, n_items=150, n_lines=9000, seed=21):
    """A synthetic Gowalla_totalCheckins.txt ('user\\ttime\\tlat\\tlon\\tloc', dataset.py:173-186):
    skewed activity so the k-core filter removes some users/items, repeated
    check-ins (duplicates with different times) and timestamp ties."""
    rng = np.random.default_rng(seed)
    w_u = 1.0 / np.arange(1, n_users + 1) ** 0.8
    w_i = 1.0 / np.arange(1, n_items + 1) ** 1.0
    u = rng.choice(n_users, n_lines, p=w_u / w_u.sum()) * 7 + 3     # sparse raw ids
    i = rng.choice(n_items, n_lines, p=w_i / w_i.sum()) * 11 + 5
    t = 1262304000 + rng.integers(0, 3000, n_lines) * 600           # 2010-01-01 + 10-minute slots (ties)
    import time as _t
    with open(path, 'w') as f:
        for a, b, c in zip(u, i, t):
            ts = _t.strftime('%Y-%m-%dT%H:%M:%SZ', _t.gmtime(int(c)))
            f.write(f'{a}\t{ts}\t30.2\t-97.7\t{b}\n')


def _skewed_ids(rng, n, n_lines, s, prefix, width):
    w = 1.0 / np.arange(1, n + 1) ** s
    ids = rng.choice(n, n_lines, p=w / w.sum())
    perm = rng.choice(10 ** width, n, replace=False)  # sparse string ids in no particular order
    return [f'{prefix}{perm[x]:0{width}d}' for x in ids]


def write_amazon_ratings(path, n_users=150, n_items=90, n_lines=9000, seed=23):
    """A synthetic ratings_Books.csv ('user,item,rating,time', dataset.py:229-244):
    string ids, ratings 1-5 (only > 3 kept), repeated pairs, timestamp ties."""
    rng = np.random.default_rng(seed)
    u = _skewed_ids(rng, n_users, n_lines, 0.8, 'A', 6)
    i = _skewed_ids(rng, n_items, n_lines, 1.0, '0', 9)
    r = rng.integers(1, 6, n_lines)
    t = 1300000000 + rng.integers(0, 2000, n_lines) * 86400
    with open(path, 'w') as f:
        for a, b, c, d in zip(u, i, r, t):
            f.write(f'{a},{b},{float(c)},{d}\n')


def write_yelp_reviews(path, n_users=140, n_items=85, n_lines=8500, seed=29):
    """A synthetic yelp_academic_dataset_review.json (one record per line,
    dataset.py:196-219): string ids, stars 1-5 (only > 3 kept), 'date' with ties."""
    import json
    rng = np.random.default_rng(seed)
    u = _skewed_ids(rng, n_users, n_lines, 0.8, 'u', 7)
    i = _skewed_ids(rng, n_items, n_lines, 1.0, 'b', 7)
    s = rng.integers(1, 6, n_lines)
    t = 1420070400 + rng.integers(0, 5000, n_lines) * 3600
    import time as _t
    with open(path, 'w') as f:
        for k, (a, b, c, d) in enumerate(zip(u, i, s, t)):
            rec = {'review_id': f'r{k}', 'user_id': a, 'business_id': b, 'stars': float(c), 'useful': 0,
                   'text': 'ok', 'date': _t.strftime('%Y-%m-%d %H:%M:%S', _t.gmtime(int(d)))}
            f.write(json.dumps(rec) + '\n')
