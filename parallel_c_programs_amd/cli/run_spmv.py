"""SpMV benchmark (ref 3-serial-optimization/spmv.c:331-367): `run_spmv dim a b c d e`.

Host path (default): prints "Time : %f s" for the naive CSR product and for the banded SIMD product, then
the compare() report — the reference's exact output. --gpu additionally times the gfx950 CSR-adaptive and
banded kernels on the same matrix (HIP events) and prints each in the reference's format ("Time : %f s" and the
compare() report against the host naive product)."""
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
            ("GPU banded, implicit columns, LDS-staged x windows", lambda: ops.spmv_banded(g.val, g.row_ptr, *dims, xg),
             m.nnz * 4 + m.n_rows * 8))
    for name, fn, bytes_ in runs:
        y = fn()
        ms = device_time_ms(fn)
        print(f"\n{name}:", flush=True)
        c_call("print_time_seconds", None, [ctypes.c_double], ms * 1e-3)
        yc = y.cpu().contiguous()
        c_call("compare", None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int], y_ref.data_ptr(), yc.data_ptr(),
               a.dim)
        print(f"({bytes_ / ms / 1e6:.1f} GB/s of compulsory traffic, {2 * m.nnz / ms / 1e6:.1f} GFLOP/s, "
              f"max |err| {(yc - y_ref).abs().max().item():.3g})", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
