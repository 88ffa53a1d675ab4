import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "psso-sac-for-powered-descent_amd")
for p in (REPO, PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


def pytest_sessionstart(session):
    # keep the in-tree HIP library current (no-op when up to date; hipcc cross-compiles)
    try:
        from pdenv import build as b
        if not b.up_to_date():
            b.build()
    except Exception as e:  # the ABI tests report the failure precisely
        print(f"[conftest] libpdenv build skipped: {e}")
