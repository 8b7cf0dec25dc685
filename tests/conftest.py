import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
ASSETS = ROOT / "assets"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on a GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def assets():
    return ASSETS


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    from parallel_c_programs_amd import _native

    _native.ops()  # must load: a GPU box without the extension is a failure, not a skip
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _chdir_tmp(tmp_path, monkeypatch):
    # tools that write ./out.bmp (reference contract) must not litter the repo
    monkeypatch.chdir(tmp_path)
    yield
