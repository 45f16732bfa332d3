import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


@pytest.fixture(scope="session")
def golden():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def built():
    """Build the engine + oracle once per session (cheap when up to date)."""
    import subprocess

    subprocess.run(["make", "-C", os.path.join(ROOT, "vortex_amd", "csrc"), "-j", "8", "-s"], check=True)
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s"], check=True)
    return True


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
