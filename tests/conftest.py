import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-lsb_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: larger sizes")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build() if not os.path.exists(oracle.LIB_PATH) else None
    return oracle


@pytest.fixture(scope="session")
def lsb_built():
    """The product library, built in-tree (fails loudly if it cannot be).

    `make` always runs: it rebuilds whatever is older than its sources, so
    the library under test is the tree's (test_library_built_from_this_tree
    checks the compiled-in source digest).  LSB_LIBRARY (another build of the
    same ABI) is used as given."""
    if not os.environ.get("LSB_LIBRARY"):
        subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
    import lsbsort
    return lsbsort


@pytest.fixture(scope="session")
def digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ref_vectors():
    with open(os.path.join(GOLDEN, "ref_print_vectors.json")) as f:
        return json.load(f)
