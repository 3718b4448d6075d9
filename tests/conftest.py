import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.hookimpl(trylast=True)   # after -m has deselected
def pytest_collection_modifyitems(config, items):
    # libvcfc.so binds to the HIP runtime already in the process (torch's
    # bundled libamdhip64.so.7 shares its soname); loaded first, it would pull
    # in ROCm's own copy and a later torch import a second runtime, in which
    # no context can be created.  A GPU run therefore imports torch before any
    # test can load the library, whatever the test order or selection.
    if any(item.get_closest_marker("gpu") for item in items):
        import torch  # noqa: F401
