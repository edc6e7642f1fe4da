import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU and the built HIP library')


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name + '.npz'))


def golden_params(d, dtype=None):
    """state_dict and grads stored as sd/<key>, grad/<key>."""
    import torch
    sd = {k[3:]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith('sd/')}
    gr = {k[5:]: d[k] for k in d.files if k.startswith('grad/')}
    if dtype is not None:
        sd = {k: v.to(dtype) for k, v in sd.items()}
    return sd, gr


@pytest.fixture(scope='session')
def cuda_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda:0')
