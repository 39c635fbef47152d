import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "spark-text-clustering_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")


@pytest.fixture(scope="session")
def ctx():
    import stc

    return stc.Context.get(0)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    return O
