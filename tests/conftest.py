import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "p2p-dhts_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: full-size property tests")


@pytest.fixture(scope="session")
def refvec():
    with open(os.path.join(GOLDEN, "reference_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def c1truth():
    with open(os.path.join(GOLDEN, "c1_truth.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def O():
    import oracle

    oracle.lib()  # fails loudly if liboracle.so was not built
    return oracle
