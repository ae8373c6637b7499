import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the kernel tests pin WHICH GEMM runs (hand-written, counted by spies): the per-shape autotune
# that may route a plain GEMM to the library is exercised by its own test (test_hip_matmul.py)
os.environ.setdefault('PADDLE_AMD_GEMM_AUTOTUNE', '0')


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def static_mode():
    import paddle
    paddle.enable_static()
    yield
    paddle.disable_static()


@pytest.fixture(autouse=True)
def _restore_paddle_device():
    """A test that switches devices (paddle.set_device) must not leak it into later tests."""
    import paddle
    dev = paddle.get_device()
    yield
    if paddle.get_device() != dev:
        paddle.set_device(dev)
