"""8-bit grayscale BMP I/O through the host C library (ref 2-mpi-region-growing/bmp.c:6-71).

read(path) -> numpy uint8 array of shape (height, width) in file row order (the reference ignores row
padding and never flips rows, so neither do we); write(path, pixels) writes the reference layout
(1078-byte header+palette, file_size = w*h + 56, 2 trailing pad bytes, all header bytes defined).
write_out_bmp(pixels) keeps the reference contract of writing ./out.bmp.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .._native import cpu_lib


def read(path) -> np.ndarray:
    lib = cpu_lib()
    w, h = ctypes.c_int(), ctypes.c_int()
    p = lib.pcmx_read_bmp_dims(os.fsencode(str(path)), ctypes.byref(w), ctypes.byref(h))
    if not p:
        raise OSError(f"cannot read BMP {path}")
    try:
        buf = (ctypes.c_ubyte * (w.value * h.value)).from_address(p)
        return np.frombuffer(buf, dtype=np.uint8).reshape(h.value, w.value).copy()
    finally:
        lib.pcmx_free(p)


def write(path, pixels) -> None:
    arr = np.ascontiguousarray(np.asarray(pixels, dtype=np.uint8))
    if arr.ndim != 2:
        raise ValueError("write: 2-D uint8 image expected")
    h, w = arr.shape
    rc = cpu_lib().pcmx_write_bmp_path(os.fsencode(str(path)), arr.ctypes.data, w, h)
    if rc != 0:
        raise OSError(f"cannot write BMP {path} (rc={rc})")


def write_out_bmp(pixels) -> None:
    """The reference's write_bmp(): always ./out.bmp."""
    write("out.bmp", pixels)
