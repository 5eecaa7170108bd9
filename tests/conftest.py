"""Test setup: import paths, the `gpu` marker, and an in-tree build of the
native library if it is missing (the .so is git-ignored)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "lds-gnn_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

_LIB = os.path.join(PKG, "ldsgnn", "libldsgnn.so")
if not os.path.exists(_LIB):
    subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc"), "-j8"], check=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")
    config.addinivalue_line("markers", "slow: long-running parity case")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def device():
    import torch
    return torch.device("cuda:0")
