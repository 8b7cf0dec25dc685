"""SpMV benchmark (ref 3-serial-optimization/spmv.c:331-367): `run_spmv dim a b c d e`.

Host path (default): prints "Time : %f s" for the naive CSR product and for the banded SIMD product, then
the compare() report — the reference's exact output. --gpu additionally times the gfx950 CSR-adaptive and
banded kernels on the same matrix (HIP events) and prints each in the reference's format ("Time : %f s", the median
of back-to-back calls, and the compare() report against the host naive product), plus its cold-cache time (median
of 5 calls each after a 1 GiB read: the 248 MB value stream of the reference config otherwise stays in the 256 MiB
Infinity Cache between calls)."""
from __future__ import annotations

import argparse
import ctypes
import sys

from ._common import c_call


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    pos = [x for x in argv if not x.startswith("--")]
    if len(pos) != 6:
        print("Usage: spmv dim a b c d e", flush=True)
        return 255
    ap = argparse.ArgumentParser(prog="run_spmv")
    for k in ("dim", "a", "b", "c", "d", "e"):
        ap.add_argument(k, type=int)
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args(argv)
    rc = c_call("pcmx_spmv_demo", ctypes.c_int, [ctypes.c_int] * 6, a.dim, a.a, a.b, a.c, a.d, a.e)
    if rc or not a.gpu:
        return rc
    import torch

    from .. import ops
    from ..utils.timing import device_time_ms

    m = ops.banded_csr(a.dim, a.a, a.b, a.c, a.d, a.e)
    x = ops.create_vector(a.dim)
    y_ref = ops.spmv(m, x)  # the host naive CSR product (the reference's r1)
    g = m.to("cuda").plan()
    xg = x.cuda()
    dims = (a.dim, a.a, a.b, a.c, a.d, a.e)
    runs = (("GPU CSR-adaptive (explicit column indices)", lambda: ops.spmv(g, xg),
             m.nnz * 8 + (m.n_rows + 1) * 8 + m.n_rows * 8),
            ("GPU banded, implicit columns, 16-B block stream + LDS x windows", lambda: ops.spmv_banded(g.val, g.row_ptr, *dims, xg),
             m.nnz * 4 + m.n_rows * 8))
    scrub = torch.empty(256 << 20, device="cuda").uniform_()  # 1 GiB, READ between cold calls (evicts the MALL)
    for name, fn, bytes_ in runs:
        y = fn()
        ms = device_time_ms(fn)
        cold = []
        for _ in range(5):
            torch.cuda.synchronize()
            # the scrub is still running when the call is enqueued: s0 fires as it ends, with the call already
            # queued behind it, so the time is the kernel's own (an idle GPU would also count the host's launch
            # latency between s0 and the kernel)
            scrub.sum()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            fn()
            s1.record()
            s1.synchronize()
            cold.append(s0.elapsed_time(s1))
        cold_ms = sorted(cold)[2]
        print(f"\n{name}:", flush=True)
        c_call("print_time_seconds", None, [ctypes.c_double], ms * 1e-3)
        yc = y.cpu().contiguous()
        c_call("compare", None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int], y_ref.data_ptr(), yc.data_ptr(),
               a.dim)
        print(f"({bytes_ / ms / 1e6:.1f} GB/s of compulsory traffic, {2 * m.nnz / ms / 1e6:.1f} GFLOP/s, "
              f"max |err| {(yc - y_ref).abs().max().item():.3g}; cold cache (after a 1 GiB read): "
              f"{cold_ms * 1e3:.1f} us = {bytes_ / cold_ms / 1e6:.1f} GB/s)", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
