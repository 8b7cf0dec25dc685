"""Shared CLI helpers: C-library calls whose stdout must interleave correctly with Python's."""
from __future__ import annotations

import ctypes
import sys

from .._native import cpu_lib


def c_call(name: str, restype, argtypes, *args):
    """Call a host C entry point, flushing both stdio layers around it so output order is preserved."""
    sys.stdout.flush()
    fn = getattr(cpu_lib(), name)
    fn.restype, fn.argtypes = restype, argtypes
    r = fn(*args)
    libc = ctypes.CDLL(None)
    libc.fflush(None)
    return r


def device_arg(ap) -> None:
    ap.add_argument("--device", default=None, help="cpu | cuda (default: cuda when a GPU is visible)")


def pick_device(name: str | None):
    import torch

    if name is None:
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(name)
