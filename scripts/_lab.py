"""Lab-build helper: compiles scripts/sgemm_lab.hip (every experimental SGEMM variant + its global tuning knobs,
which the production libpcmx_hip does not carry) into build/lab/libpcmx_sgemm_lab.so and calls it on torch tensors."""
import ctypes
import subprocess
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "scripts" / "sgemm_lab.hip"
SO = ROOT / "build" / "lab" / "libpcmx_sgemm_lab.so"
_lib = None


def sgemm_lab() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not SO.exists() or SO.stat().st_mtime < SRC.stat().st_mtime:
            SO.parent.mkdir(parents=True, exist_ok=True)
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950",
                            f"-I{ROOT / 'csrc/include'}", f"-I{ROOT / 'csrc/runtime'}", str(SRC), "-o", str(SO)],
                           check=True)
        torch.cuda.init()  # one HIP runtime: the lab library binds to the one torch loaded
        _lib = ctypes.CDLL(str(SO))
        _lib.pcmx_sgemm_lab_variant.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 6 + [ctypes.c_float] * 2 + \
            [ctypes.c_int, ctypes.c_void_p]
        _lib.pcmx_sgemm_lab_set_tuning.argtypes = [ctypes.c_int, ctypes.c_int]
    return _lib


def set_tuning(tile_order: int, k0_diag: int) -> None:
    assert sgemm_lab().pcmx_sgemm_lab_set_tuning(tile_order, k0_diag) == 0


def sgemm(a: torch.Tensor, b: torch.Tensor, variant: int, out: torch.Tensor | None = None) -> torch.Tensor:
    m, k = a.shape
    n = b.shape[1]
    c = torch.empty(m, n, device=a.device) if out is None else out
    rc = sgemm_lab().pcmx_sgemm_lab_variant(a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, a.stride(0), b.stride(0),
                                            c.stride(0), 1.0, 0.0, variant,
                                            torch.cuda.current_stream(a.device).cuda_stream)
    if rc:
        raise RuntimeError(f"lab sgemm variant {variant}: rc {rc}")
    return c


_libs = {}


def lab_lib(name: str, entry: str) -> ctypes.CDLL:
    """Build scripts/<name>.hip into build/lab/lib<name>.so (on the box that runs it) and bind `entry` with the
    variant-launcher signature (A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, variant, stream)."""
    if name not in _libs:
        src = ROOT / "scripts" / f"{name}.hip"
        so = ROOT / "build" / "lab" / f"lib{name}.so"
        if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
            so.parent.mkdir(parents=True, exist_ok=True)
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950",
                            f"-I{ROOT / 'csrc/include'}", f"-I{ROOT / 'csrc/runtime'}", str(src), "-o", str(so)],
                           check=True)
        torch.cuda.init()
        lib = ctypes.CDLL(str(so))
        fn = getattr(lib, entry)
        fn.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 6 + [ctypes.c_float] * 2 + [ctypes.c_int, ctypes.c_void_p]
        _libs[name] = fn
    return _libs[name]


def sgemm_dr(a: torch.Tensor, b: torch.Tensor, variant: int, out: torch.Tensor | None = None) -> torch.Tensor:
    fn = lab_lib("sgemm_dr_lab", "pcmx_sgemm_dr_lab_variant")
    m, k = a.shape
    n = b.shape[1]
    c = torch.empty(m, n, device=a.device) if out is None else out
    rc = fn(a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, a.stride(0), b.stride(0), c.stride(0), 1.0, 0.0, variant,
            torch.cuda.current_stream(a.device).cuda_stream)
    if rc:
        raise RuntimeError(f"dr lab sgemm variant {variant}: rc {rc}")
    return c
