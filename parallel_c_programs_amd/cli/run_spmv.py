"""SpMV benchmark (ref 3-serial-optimization/spmv.c:331-367): `run_spmv dim a b c d e`.

Host path (default): prints "Time : %f s" for the naive CSR product and for the banded SIMD product, then
the compare() report — the reference's exact output. --gpu additionally times the gfx950 CSR-adaptive and
banded kernels on the same matrix and checks them against the host result."""
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
    y_ref = ops.spmv(m, x)
    g = m.to("cuda").plan()
    xg = x.cuda()
    y = ops.spmv(g, xg)
    ms = device_time_ms(lambda: ops.spmv(g, xg))
    err = (y.cpu() - y_ref).abs().max().item()
    gbs = (m.nnz * 8 + (m.n_rows + 1) * 8 + m.n_rows * 8) / ms / 1e6
    print(f"GPU CSR-adaptive: {ms * 1e-3:f} s ({gbs:.1f} GB/s, max |err| {err:.3g})", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
