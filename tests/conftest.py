import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfvc on cuda:0)")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fastvideocodec_amd import _lib
    _lib.load()
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def seeded_sd():
    from fastvideocodec_amd.weights import seeded_torch_state_dict
    return seeded_torch_state_dict()
