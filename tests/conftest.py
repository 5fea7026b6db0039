import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "asr-transformer_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(autouse=True)
def _reset_dropout_seed_offset(request):
    """A Trainer step leaves the device-resident dropout seed offset at its step count (asrx_set_seed_offset);
    kernel tests compare keep bits with rng_ref at offset 0, so every GPU test starts from offset 0."""
    if request.node.get_closest_marker("gpu") is not None:
        import torch
        if torch.cuda.is_available():
            from asrx import kernels as K
            K.set_seed_offset(0)
            torch.cuda.synchronize()
    yield


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
