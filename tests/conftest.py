import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


@pytest.hookimpl(tryfirst=True)  # before xdist's own (tryfirst too; later-registered runs first)
def pytest_cmdline_main(config):
    """The CPU suite (`-m "not gpu"`) runs on 4 xdist workers unless `-n` is
    given or DISSEM_TEST_SERIAL=1: its tests are process-isolated by design
    (per-test fabric keys, ports from the OS) and pass 10 of 10 times at -n 4
    (profiles/r6_determinism/). GPU runs stay in one process."""
    opt = config.option
    if hasattr(config, "workerinput") or os.environ.get("PYTEST_XDIST_WORKER"):
        return None  # an xdist worker itself
    if ("not gpu" not in (getattr(opt, "markexpr", "") or "") or os.environ.get("DISSEM_TEST_SERIAL") == "1"
            or not hasattr(opt, "numprocesses") or opt.numprocesses or (os.cpu_count() or 1) < 4
            or getattr(opt, "collectonly", False)):
        return None
    opt.numprocesses = 4
    return None


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
