import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def kat():
    return json.load(open(os.path.join(GOLDEN, "kat.json")))["cases"]


@pytest.fixture(scope="session")
def batches():
    return json.load(open(os.path.join(GOLDEN, "batches.json")))


@pytest.fixture(scope="session")
def oracle():
    from oracle.pyoracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def gpu():
    """The product library on a visible MI355X; fails (not skips) without one."""
    import torch
    import liblcb_amd
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    assert liblcb_amd.lib().lcb_hash_gpu_device_count() > 0
    return liblcb_amd
