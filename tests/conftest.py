import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU cross-checks")


GOLDEN = os.path.join(ROOT, "tests", "golden")


def golden_cases():
    import json
    with open(os.path.join(GOLDEN, "index.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    return oracle.lib()
