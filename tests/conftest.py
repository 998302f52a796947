import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
for p in (ROOT, os.path.join(ROOT, 'oracle')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP device); run with -m gpu')
    config.addinivalue_line('markers', 'slow: long-running parity case')


def golden(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.skip(f'golden fixture {name} not generated')
    return np.load(path)


@pytest.fixture(scope='session')
def gpu():
    """Product package on a real GPU: fails (not skips) if the HIP library is missing."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    import nngp_amd
    nngp_amd.lib()
    return nngp_amd
