"""Test configuration.

Markers:
  gpu -- needs an MI355X (runs the HIP library through its C ABI).
Everything else runs on CPU in the build container.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ska-sdp-func_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: requires an AMD Instinct GPU (MI355X) and the HIP build")


@pytest.fixture(scope="session")
def device():
    """The GPU device; fails (does not skip) if the GPU path is unavailable."""
    import torch

    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch.device("cuda:0")
