import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.path.join(ROOT, "tests") not in sys.path:
    sys.path.insert(0, os.path.join(ROOT, "tests"))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")
    # before collection: test modules import cilium_amd, which refuses a library
    # built from other sources (the session fixture below keeps the same guarantee)
    import __graft_entry__
    __graft_entry__.build()


@pytest.fixture(scope="session", autouse=True)
def _built():
    # build() recompiles only when the in-tree library is missing or was built
    # from other sources (its gf_build_id() digest), so a test run always uses a
    # binary of the tree it tests
    import __graft_entry__
    __graft_entry__.build()
    yield
