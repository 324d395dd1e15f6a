import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device and the built extension")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _restore_deterministic_mode():
    """A test that switches the kernels to deterministic mode must not leak it into the next
    one (deterministic mode refuses the atomic weight-gradient paths some kernel tests use)."""
    yield
    if "perceiver_io_amd.ops" in sys.modules:
        from perceiver_io_amd import ops

        if ops.deterministic():
            ops.set_deterministic(False)
