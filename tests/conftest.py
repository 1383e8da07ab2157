"""Test configuration.

Markers:
  gpu — needs a HIP device (MI355X); run with `pytest -m gpu` on the GPU box.
GPU tests are never skipped silently: without a device they fail loudly
(the engine has no CPU fallback).  Everything else runs on CPU (oracle vs golden fixtures, host logic, C-ABI
symbol checks, multi-process gloo tests).
"""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a HIP GPU (MI355X)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
