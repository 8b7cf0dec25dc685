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


def cli_env(**extra) -> dict:
    """Environment for `python -m parallel_c_programs_amd.cli.*` subprocesses run from a tmp cwd."""
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.update(extra)
    return env


def run_cli(module: str, *args, check=True, timeout=600, **env):
    import subprocess

    return subprocess.run([sys.executable, "-m", f"parallel_c_programs_amd.cli.{module}", *map(str, args)],
                          capture_output=True, text=True, check=check, timeout=timeout, env=cli_env(**env))


@pytest.fixture(autouse=True)
def _chdir_tmp(tmp_path, monkeypatch):
    # tools that write ./out.bmp (reference contract) must not litter the repo
    monkeypatch.chdir(tmp_path)
    yield
