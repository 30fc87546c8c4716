import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'oracle'))
GOLDEN = ROOT / 'tests' / 'golden'


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device) and libxagents_hip.so')


@pytest.fixture(scope='session')
def device():
    import torch

    if not torch.cuda.is_available():
        pytest.fail('gpu test selected but no HIP device is visible')
    from xagents_amd import _lib

    _lib.load()  # raises loudly if the extension is missing
    import os
    if os.environ.get('XA_LIB'):
        # (diagnostic A/B only) run the GPU tests against a variant build of the library
        # (tools/build_variant.py); the driver's runs never set it
        _lib._lib = _lib.load(os.environ['XA_LIB'])
    return torch.device('cuda')


@pytest.fixture(scope='session')
def golden():
    import numpy as np

    def load(name):
        return np.load(GOLDEN / name, allow_pickle=False)

    return load
