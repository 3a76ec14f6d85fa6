import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu on the GPU box")


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    if not os.path.exists(pyoracle.ORACLE_SO):
        pyoracle.build()
    return pyoracle.Oracle()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    return load


@pytest.fixture(scope="session")
def bp():
    """The product library, loaded and with a GPU present (gpu tests only)."""
    import cudabulletproof_amd as m
    m.build()
    m.require_gpu()
    return m
