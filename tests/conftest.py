import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ibond-flex_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_fb():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden_fb.json")) as f:
        return json.load(f)
