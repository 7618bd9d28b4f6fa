import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP kernels)')


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope='session')
def gpu():
    if not gpu_available():
        pytest.fail('GPU test selected but no GPU is visible (run with -m "not gpu" on CPU hosts)')
    import torch
    return torch.device('cuda:0')
