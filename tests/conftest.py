import os
import sys

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


def pytest_collection_modifyitems(config, items):
    # A -m gpu run on a box without a GPU should fail loudly, not skip silently;
    # a CPU run (-m "not gpu") never collects them.
    pass
