import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hybrid-genome-assembler_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def hga_mod():
    import hga
    return hga


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    return oracle


@pytest.fixture(scope="session")
def gpu_ctx():
    import hga
    ctx = hga.Ctx(int(os.environ.get("HGA_DEVICE", "0")))
    yield ctx
    ctx.close()
