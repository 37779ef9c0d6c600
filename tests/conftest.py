import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "siril-0.9_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def gpu_ctx():
    # torch (device buffers for the device-resident tests) brings its own HIP runtime; it
    # must initialise the GPU before libsirilgpu's runtime does, as bench.py does
    import torch
    torch.cuda.init()
    torch.zeros(1, device="cuda")
    import sirilgpu
    ctx = sirilgpu.Context()
    yield ctx
    ctx.close()
