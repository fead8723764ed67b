import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) device')
    config.addinivalue_line('markers', 'slow: long-running')


@pytest.fixture(scope='session', autouse=True)
def _threads():
    import torch
    torch.set_num_threads(4)   # the fixtures were generated at 4 threads (src/cli.py:108)
    yield


def load_golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False)
