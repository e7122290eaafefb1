"""Generate tests/golden/config_rows.json from the reference's config tables
(config.py:1-527): for each of its five getters, the number of rows and the rows
whose model is on the hot path (LightGCN / IGCN / NGCF / IMF / IMCGAE), keyed by their index.

Run:  python tests/golden/make_config_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, '/root/reference')
import config as ref_config  # noqa: E402

ON_PATH = {'LightGCN', 'IGCN', 'NGCF', 'IMF', 'IMCGAE'}


def main():
    out = {}
    for fn in ['get_gowalla_config', 'get_yelp_config', 'get_amazon_config', 'get_alibaba_config', 'get_ml_config']:
        rows = getattr(ref_config, fn)('DEVICE')
        out[fn] = {'n_rows': len(rows),
                   'rows': {str(k): [d, m, t] for k, (d, m, t) in enumerate(rows) if m['name'] in ON_PATH}}
    path = os.path.join(HERE, 'config_rows.json')
    with open(path, 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print('wrote', path, {k: (v['n_rows'], sorted(v['rows'], key=int)) for k, v in out.items()})


if __name__ == '__main__':
    main()
