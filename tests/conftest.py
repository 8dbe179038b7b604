import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long running")


@pytest.fixture(scope="session")
def pa():
    import parsec_amd

    if not parsec_amd.native_available():
        from parsec_amd import _build

        _build.build()
        import importlib

        parsec_amd = importlib.reload(parsec_amd)
    parsec_amd.require_native()
    return parsec_amd
