"""Golden splits for the raw-log loaders: the REFERENCE's YelpDataset and
AmazonDataset (dataset.py:192-255, i.e. remove_sparse_ui + update_user_inter_lists
+ generate_data, dataset.py:66-114) run on synthetic files written by
ml_like.py.  Output: tests/golden/ingest_{amazon,yelp}.npz (data only).
Run from this directory: python make_ingest_golden.py"""
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'
sys.path.insert(0, HERE)
import ml_like  # noqa: E402


def main():
    os.environ['TZ'] = 'UTC'  # the reference parses Yelp dates with time.mktime (local time)
    time.tzset()
    sys.path.insert(0, REF)
    import dataset as ref_dataset
    cases = [('amazon', 'AmazonDataset', 'ratings_Books.csv', ml_like.write_amazon_ratings),
             ('yelp', 'YelpDataset', 'yelp_academic_dataset_review.json', ml_like.write_yelp_reviews)]
    for tag, cls, fname, writer in cases:
        with tempfile.TemporaryDirectory() as tmp:
            writer(os.path.join(tmp, fname))
            out = {}
            for k in (5, 10):
                ds = getattr(ref_dataset, cls)({'name': cls, 'path': tmp, 'device': 'cpu', 'min_inter': k,
                                                'split_ratio': [0.8, 0.1, 0.1]})
                out[f'k{k}_n'] = np.array([ds.n_users, ds.n_items], np.int64)
                for split in ['train', 'val', 'test']:
                    data = getattr(ds, split + '_data')
                    out[f'k{k}_{split}_ptr'] = np.cumsum([0] + [len(x) for x in data]).astype(np.int64)
                    out[f'k{k}_{split}_items'] = np.array(sum(data, []), dtype=np.int64)
            np.savez_compressed(os.path.join(HERE, f'ingest_{tag}.npz'), **out)
            print(tag, {k: v.tolist() for k, v in out.items() if k.endswith('_n')})


if __name__ == '__main__':
    main()
