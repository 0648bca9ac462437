import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libromis_amd.so; run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def abi_lib():
    """libromis_amd.so loaded for its host-only entry points (no GPU calls)."""
    from romis_amd import _abi, build
    build.build()
    return _abi.load_library()
