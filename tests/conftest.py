import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


@pytest.fixture(scope="session")
def g():
    import __graft_entry__ as ge
    lib = os.path.join(ROOT, "go-raytracing_amd", "lib")
    if not (os.path.exists(os.path.join(lib, "librtgpu.so")) and os.path.exists(os.path.join(lib, "librtscene.so"))):
        ge.build()
    return ge.load_package()


@pytest.fixture(scope="session")
def O():
    from oracle import oracle_py
    oracle_py.lib()
    return oracle_py


@pytest.fixture(scope="session")
def ctx(g):
    c = g.Context(0)
    yield c
    c.close()
