"""North-star SGEMM CLI: C = A @ B, fp32, on one MI355X (ancestor: matrix_multiply, ref 1-introduction/matrix.c:63-81).

    run_sgemm [N] [--m M --k K] [--precision fp32|bf16x6] [--steps S --warmup W] [--compare] [--seed X]

  --precision fp32    the native f32-MFMA kernel (sgemm.hip, production variant 17: the bench's `value`)
  --precision bf16x6  fp32 accuracy on the bf16 matrix cores (sgemm_x6.hip, variant 20: exact 3-way operand split,
                      6 piece products)
  --compare           also time hipBLASLt (torch.matmul) on the same operands, identically, and print both errors

Prints the reference's "Time : %f s" line (mean per product) and one JSON line: TFLOPS, ms, the max relative error of
a row sample against the fp64 product (normalised by the largest reference entry, as bench.py), and the comparison.
Shapes that are not tile-aligned are padded by ops.sgemm (the timed product runs on the padded operands' kernel).
Without a GPU the host C GEMM backend runs (fp32 only)."""
from __future__ import annotations

import argparse
import json

import torch

from .. import ops
from ..utils.timing import print_time

VARIANTS = {"fp32": 17, "bf16x6": 20}


def _timed(fn, steps: int, warmup: int, cuda: bool) -> float:
    for _ in range(warmup):
        fn()
    if not cuda:
        import time

        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        return (time.perf_counter() - t0) / steps
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / 1e3 / steps


def _err(c: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> float:
    rows = torch.arange(0, a.shape[0], max(1, a.shape[0] // 8), device=a.device)
    ref = a[rows].double() @ b.double()
    return ((c[rows].double() - ref).abs().max() / ref.abs().max().clamp_min(1e-300)).item()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run_sgemm", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("n", nargs="?", type=int, default=8192, help="N (M = K = N unless given)")
    ap.add_argument("--m", type=int, default=0)
    ap.add_argument("--k", type=int, default=0)
    ap.add_argument("--precision", choices=tuple(VARIANTS), default="fp32")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--compare", action="store_true", help="time hipBLASLt (torch.matmul) the same way")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default=None, help="cuda (default with a GPU) or cpu")
    a = ap.parse_args(argv)
    dev = torch.device(a.device or ("cuda" if torch.cuda.is_available() else "cpu"))
    cuda = dev.type == "cuda"
    if not cuda and a.precision != "fp32":
        ap.error("--precision bf16x6 needs the GPU (the host backend is fp32)")
    n, m, k = a.n, a.m or a.n, a.k or a.n
    g = torch.Generator(device=dev).manual_seed(a.seed)
    A = torch.rand(m, k, device=dev, generator=g) * 2 - 1
    B = torch.rand(k, n, device=dev, generator=g) * 2 - 1
    variant = VARIANTS[a.precision] if cuda else -1
    out = {}

    def ours():
        out["c"] = ops.sgemm(A, B, variant=variant)

    secs = _timed(ours, a.steps, a.warmup, cuda)
    flop = 2.0 * m * n * k
    print_time(secs)
    line = {"workload": "sgemm", "m": m, "n": n, "k": k, "precision": a.precision, "device": dev.type,
            "kernel": f"variant {variant}" if cuda else "host C backend", "ms": round(secs * 1e3, 4),
            "tflops": round(flop / secs / 1e12, 3), "max_rel_err_vs_fp64": _err(out["c"], A, B)}
    if a.compare and cuda:
        ref = {}
        t_ref = _timed(lambda: ref.__setitem__("c", torch.matmul(A, B)), a.steps, a.warmup, cuda)
        line.update({"hipblaslt_torch_matmul_tflops": round(flop / t_ref / 1e12, 3),
                     "hipblaslt_max_rel_err_vs_fp64": _err(ref["c"], A, B),
                     "speedup_vs_hipblaslt": round(t_ref / secs, 4)})
    print(json.dumps(line), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
