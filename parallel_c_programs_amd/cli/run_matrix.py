"""matrix demo (ref 1-introduction/matrix.c:117-225): matrix_t create/print/multiply/resize walkthrough.

--compat reproduces the reference's inverted is_sparse (bug B1) so the printed lines match
the reference binary; the default prints the corrected result.

--gemm N (beyond the reference's 2x2 walkthrough): the same matrix_multiply at N x N x N on random operands,
through the backend matrix_t dispatches to (the f32-MFMA kernel on a GPU, the threaded host GEMM otherwise):
prints the mean time of --reps calls after a warm-up, the TFLOP/s and the max relative error of EVERY element
against an fp64 product, and exits 1 when that error exceeds 1e-5 (the bench's limit).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import time

from ._common import c_call

REL_ERR_LIMIT = 1e-5


def gemm_check(n: int, reps: int = 5, device: str | None = None, seed: int = 0) -> dict:
    """C = A @ B (f32, n^3) through ops.sgemm, timed and checked element by element against fp64."""
    import torch

    from .. import ops

    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    g = torch.Generator(device=dev).manual_seed(seed)
    a = torch.rand(n, n, device=dev, generator=g) - 0.5
    b = torch.rand(n, n, device=dev, generator=g) - 0.5
    c = ops.sgemm(a, b)  # warm-up (and the checked result)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        c = ops.sgemm(a, b)
    sync()
    ms = (time.perf_counter() - t0) / reps * 1e3
    ref = a.double() @ b.double()
    err = ((c.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-300)).item()
    return {"n": n, "device": str(dev), "ms": round(ms, 4), "tflops": round(2.0 * n ** 3 / ms / 1e9, 2),
            "max_rel_err_vs_fp64": err, "check_passed": err <= REL_ERR_LIMIT}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run_matrix")
    ap.add_argument("--compat", action="store_true", help="keep the reference's is_sparse bug (B1)")
    ap.add_argument("--gemm", type=int, default=0, metavar="N", help="time + check an N x N x N f32 multiply")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--device", default=None, help="cuda (default when a GPU is visible) or cpu")
    a = ap.parse_args(argv)
    if a.gemm > 0:
        r = gemm_check(a.gemm, a.reps, a.device)
        print(json.dumps(r), flush=True)
        return 0 if r["check_passed"] else 1
    return c_call("pcmx_matrix_demo", ctypes.c_int, [ctypes.c_int], int(a.compat))


if __name__ == "__main__":
    raise SystemExit(main())
