"""Raw-log ingestion timed against the reference's own loader (host only, no GPU).

A synthetic Gowalla check-in file (tests/golden/ml_like.write_checkins, the format of
dataset.py:173-186) is read by igr.dataset.GowallaDataset and, when the reference is present
(/root/reference, this container only), by the reference's GowallaDataset (dataset.py:167-189:
k-core filter, earliest time per pair, per-user time-ordered split).  Both must produce the same
splits; prints one JSON line with the two times.
    python scripts/bench_ingest.py [--lines 2000000]"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'inductive-recommendation_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
REF = '/root/reference'


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lines', type=int, default=2_000_000)
    ap.add_argument('--users', type=int, default=40_000)
    ap.add_argument('--items', type=int, default=60_000)
    args = ap.parse_args()
    os.environ['TZ'] = 'UTC'  # the reference parses dates with time.mktime (local time)
    time.tzset()
    import ml_like
    from igr import dataset as D
    cfg = {'name': 'GowallaDataset', 'device': 'cpu', 'min_inter': 10, 'split_ratio': [0.8, 0.1, 0.1]}
    out = {'file': 'synthetic Gowalla_totalCheckins.txt', 'lines': args.lines, 'min_inter': 10}
    with tempfile.TemporaryDirectory() as tmp:
        ml_like.write_checkins(os.path.join(tmp, 'Gowalla_totalCheckins.txt'), n_users=args.users, n_items=args.items,
                               n_lines=args.lines)
        t0 = time.perf_counter()
        ours = D.GowallaDataset(dict(cfg, path=tmp))
        out['igr_s'] = time.perf_counter() - t0
        out['n_users'], out['n_items'] = ours.n_users, ours.n_items
        out['train_interactions'] = int(sum(len(x) for x in ours.train_data))
        if os.path.isdir(REF):
            sys.path.insert(0, REF)
            import dataset as ref_dataset
            t0 = time.perf_counter()
            ref = ref_dataset.GowallaDataset(dict(cfg, path=tmp))
            out['reference_s'] = time.perf_counter() - t0
            same = (ref.n_users, ref.n_items) == (ours.n_users, ours.n_items)
            for split in ('train_data', 'val_data', 'test_data'):
                theirs, mine = getattr(ref, split), getattr(ours, split)
                same = same and [list(map(int, x)) for x in theirs] == [list(map(int, x)) for x in mine]
            out['identical_splits'] = bool(same)
            out['speedup'] = out['reference_s'] / out['igr_s']
    print(json.dumps(out))


if __name__ == '__main__':
    main()
