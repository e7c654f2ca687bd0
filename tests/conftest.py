import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams-ts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def engine():
    # torch's HIP runtime first (tests that hand torch device buffers to the
    # engine need it to see the device), then the engine's
    import torch

    if torch.cuda.is_available():
        torch.cuda.init()
    import zsamd

    return zsamd.Engine(0)
