import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "fast-livo-noted_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: full-size (1M/10M map) cases")


@pytest.fixture(scope="session")
def built():
    """Build the oracle (CPU) and make sure the HIP library exists."""
    import oracle

    oracle.build()
    import build as livo_build

    livo_build.build()
    return True


@pytest.fixture(scope="session")
def map100k():
    from livo_amd import synth

    return synth.make_map(100_000)


@pytest.fixture(scope="session")
def tree100k(built, map100k):
    import oracle

    return oracle.Tree(map100k)


@pytest.fixture(scope="session")
def gpu_ctx(built):
    import livo_amd
    from livo_amd import synth

    ctx = livo_amd.Context(0, t_LI=synth.T_LI, max_iterations=4)
    yield ctx
    ctx.close()
