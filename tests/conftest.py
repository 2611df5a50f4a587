import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "iterative-closest-point_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: minutes-long CPU test")


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    oracle_py.lib()
    return oracle_py


@pytest.fixture(scope="session")
def icp_lib():
    """The product C-ABI library; built on demand (hipcc cross-compiles without a GPU)."""
    import subprocess
    import icp_amd
    if not os.path.exists(icp_amd.LIB_PATH):
        subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True)
    icp_amd.lib()
    return icp_amd


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "traces.json")) as f:
        return json.load(f)
