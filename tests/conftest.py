import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu() -> bool:
    if os.path.exists("/dev/kfd"):
        try:
            import torch
            return torch.cuda.device_count() > 0
        except Exception:
            return False
    return False


HAS_GPU = _has_gpu()


def pytest_collection_modifyitems(config, items):
    if HAS_GPU:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def native_built():
    """Build every native target once per session (CMake, in-tree)."""
    from dynolog_amd import _native
    _native.ensure_built(gpu=True)
    return _native
