"""Test configuration.

Markers:
  gpu -- needs a real MI355X (run on the GPU box with `pytest -m gpu`); these
         tests call the HIP kernels through the C-ABI and compare them with the
         CPU oracle.  Everything else runs on the CPU in a few minutes.
"""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
TESTS = Path(__file__).resolve().parent
if str(TESTS) not in sys.path:
    sys.path.insert(0, str(TESTS))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def renderer():
    import torch
    from sdf3d_amd import Renderer
    from sdf3d_amd import build as b
    # a fresh checkout builds the in-tree library and host program first (no-op
    # when they are up to date)
    b.build_library(verbose=False)
    b.build_example(verbose=False)
    # GPU tests must not pass silently without a device: fail, do not skip.
    assert torch.cuda.is_available(), "gpu test run without a visible HIP device"
    return Renderer("cuda:0")
