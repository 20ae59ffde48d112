import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library through its C ABI)")
    config.addinivalue_line("markers", "slow: large-size CPU cases")


def _have_gpu():
    try:
        import dvbt2ll
        return dvbt2ll.lib().dvbt2ll_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    # torch's HIP runtime (used by the stream / device-buffer tests) is brought up before the
    # library's own, as in bench.py and the INTEGRATION.md examples
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    if not _have_gpu():
        pytest.fail("gpu-marked test but no GPU / HIP library available")
    return True
