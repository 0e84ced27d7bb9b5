import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and nex_amd/libnexg.so")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.lib()
    return o


@pytest.fixture(scope="session")
def engine():
    """The HIP engine on cuda:0. GPU tests FAIL (not skip) if the library is
    missing on a GPU box: there is no fallback to hide behind."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU in this environment")
    from nex_amd.engine import Engine
    return Engine(0)
