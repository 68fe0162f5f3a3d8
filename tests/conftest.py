import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU test")


GOLDEN = os.path.join(REPO, "tests", "golden")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
