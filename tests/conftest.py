"""Test configuration: markers and import paths.

`-m "not gpu"`: oracle vs golden vectors, host logic, C-ABI symbol checks (CPU only).
`-m gpu`: HIP parity tests through the C ABI (need an MI355X).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "speech-denoising-diffusion-model-2_amd")
for p in (REPO, PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test without a visible HIP device")
    return torch
