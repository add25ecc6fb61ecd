import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: multi-second test")


@pytest.fixture(scope="session")
def core():
    import distributed_llm_dissemination_amd as dl

    dl._core.set_log_level(3)
    return dl._core


@pytest.fixture(scope="session")
def gpu(core):
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a GPU")
    torch.cuda.set_device(0)
    return core
