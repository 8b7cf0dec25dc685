"""Loader for the in-tree native libraries.

* ``_C.so``            registers ``torch.ops.pcmx.*`` (the MI355X kernels, dispatch key CUDA == HIP device)
* ``lib/libpcmx_cpu.so`` host C library (BMP, matrix_t, SpMV, histogram, oracles) via ctypes
* ``lib/libpcmx_hip.so`` the C ABI of the kernels (device info, host-array GEMM backend) via ctypes

GPU paths never fall back silently: if a GPU is visible and the extension is missing, ``ops()`` raises.
"""
from __future__ import annotations

import ctypes
import importlib
import os
import threading
from pathlib import Path

import torch

PKG_DIR = Path(__file__).resolve().parent
LIB_DIR = PKG_DIR / "lib"
_lock = threading.Lock()
_state = {"ops": None, "cpu": None, "hip": None, "err": None}


class NativeMissing(RuntimeError):
    pass


def _try_build():
    if os.environ.get("PCMX_NO_AUTOBUILD"):
        return
    from . import _build

    _build.build_all()


def ops():
    """Return ``torch.ops.pcmx`` after loading ``_C.so`` (raises if it cannot be loaded)."""
    with _lock:
        if _state["ops"] is not None:
            return _state["ops"]
        try:
            importlib.import_module(f"{__package__}._C")
        except ImportError as e:  # first use in a fresh checkout: build in-tree, then retry once
            try:
                _try_build()
                importlib.import_module(f"{__package__}._C")
            except Exception as e2:  # pragma: no cover - surfaced to the caller
                _state["err"] = e2
                raise NativeMissing(f"pcmx native extension unavailable: {e!r} / {e2!r}") from e2
        _state["ops"] = torch.ops.pcmx
        return _state["ops"]


def native_available() -> bool:
    try:
        ops()
        return True
    except NativeMissing:
        return False


def cpu_lib() -> ctypes.CDLL:
    with _lock:
        if _state["cpu"] is None:
            so = LIB_DIR / "libpcmx_cpu.so"
            if not so.exists():
                _try_build()
            _state["cpu"] = _declare_cpu(ctypes.CDLL(str(so)))
        return _state["cpu"]


def hip_lib() -> ctypes.CDLL:
    with _lock:
        if _state["hip"] is None:
            so = LIB_DIR / "libpcmx_hip.so"
            if not so.exists():
                _try_build()
            lib = ctypes.CDLL(str(so))
            lib.pcmx_device_count.restype = ctypes.c_int
            lib.pcmx_sgemm_host_arrays.restype = ctypes.c_int
            lib.pcmx_print_device_info.argtypes = [ctypes.c_int]
            lib.pcmx_register_gemm_backend.argtypes = [ctypes.c_longlong]
            _state["hip"] = lib
        return _state["hip"]


P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F = ctypes.c_float
D = ctypes.c_double


def _declare_cpu(lib: ctypes.CDLL) -> ctypes.CDLL:
    sig = {
        "pcmx_read_bmp_dims": (P, [ctypes.c_char_p, ctypes.POINTER(I), ctypes.POINTER(I)]),
        "pcmx_write_bmp_path": (I, [ctypes.c_char_p, P, I, I]),
        "write_bmp": (None, [P, I, I]),
        "pcmx_free": (None, [P]),
        "pcmx_sgemm_host": (None, [P, P, P, I, I, I]),
        "pcmx_sgemm_naive": (None, [P, P, P, I, I, I]),
        "pcmx_histeq_serial": (None, [P, P, I]),
        "pcmx_histeq_omp": (None, [P, P, I, I]),
        "pcmx_histeq_pthreads": (None, [P, P, I, I]),
        "pcmx_histogram_u8": (None, [P, I, P]),
        "pcmx_transfer_function": (None, [P, I, P]),
        "pcmx_vmul_host": (None, [P, P, P, LL]),
        "pcmx_vadd_omp": (None, [P, P, P, LL, I]),
        "pcmx_axpy_omp": (None, [F, P, P, LL, I]),
        "pcmx_dot_omp": (D, [P, P, LL, I]),
        "pcmx_sum_omp": (D, [P, LL, I]),
        "pcmx_region2d_serial": (LL, [P, I, I, P, I, I, P]),
        "pcmx_region3d_serial": (LL, [P, I, I, I, I, I, P]),
        "pcmx_create_data": (None, [P, I]),
        "pcmx_create_data_hash": (None, [P, I, ctypes.c_uint]),
        "pcmx_raycast_serial": (None, [P, P, I, I, P]),
        "pcmx_spmv_csr_omp": (None, [I, P, P, P, P, P]),
        "pcmx_band_ranges": (None, [I, I, I, I, I, I, I, P, P]),
        "pcmx_powerlaw_row_counts": (LL, [I, LL, D, ctypes.c_ulonglong, P]),
        "pcmx_powerlaw_fill": (None, [I, I, P, ctypes.c_ulonglong, P, P]),
        "pcmx_powerlaw_fill_rows": (None, [I, I, I, P, ctypes.c_ulonglong, P, P]),
        "pcmx_wtime": (D, []),
        "pcmx_omp_max_threads": (I, []),
        "diag_count": (I, [I, I]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def ptr(t: torch.Tensor) -> int:
    """Raw data pointer of a contiguous CPU tensor (for ctypes calls)."""
    assert t.is_contiguous(), "ctypes calls need contiguous tensors"
    return t.data_ptr()
