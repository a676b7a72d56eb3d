import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through librl.so on the GPU)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


def pytest_collection_modifyitems(config, items):
    # GPU tests are expensive per process: keep them in one process, in file order.
    pass
