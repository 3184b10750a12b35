"""Test configuration: ``gpu`` marker + in-tree native build.

``pytest -m "not gpu"`` runs everything on the CPU (host mirror, gloo
multi-process tests); ``pytest -m gpu`` runs the MI355X kernel tests.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X / gfx950)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Make sure analyzer_amd/_C is built in-tree (compiles for gfx950 + host)."""
    from analyzer_amd import build_ext

    build_ext.build(jobs=4)
    yield


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    return torch.device("cuda:0")
