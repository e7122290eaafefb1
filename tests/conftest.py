import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'inductive-recommendation_amd')
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')
CASES = ['toy', 'uni', 'pow']


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the HIP C-ABI library)')


@pytest.fixture(params=CASES)
def golden(request):
    import numpy as np
    with np.load(os.path.join(GOLDEN, request.param + '.npz')) as z:
        fx = {k: z[k] for k in z.files}
    fx['_name'] = request.param
    return fx
