"""North-star config 1: vector add + dot of 1e7 f32 on the CPU with OpenMP (`run_vecops [n] [threads] [reps]`).
--gpu also times the gfx950 streaming kernels."""
from __future__ import annotations

import argparse
import ctypes

from ._common import c_call


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run_vecops")
    ap.add_argument("n", type=int, nargs="?", default=10_000_000)
    ap.add_argument("threads", type=int, nargs="?", default=0)
    ap.add_argument("reps", type=int, nargs="?", default=10)
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args(argv)
    rc = c_call("pcmx_vecops_demo", ctypes.c_int, [ctypes.c_longlong, ctypes.c_int, ctypes.c_int],
                a.n, a.threads, a.reps)
    if rc or not a.gpu:
        return rc
    import torch

    from .. import ops
    from ..utils.timing import device_time_ms

    x = torch.empty(a.n, device="cuda")
    y = torch.empty(a.n, device="cuda")
    ops.rand_uniform_(x, 1)
    ops.rand_uniform_(y, 2)
    t_add = device_time_ms(lambda: ops.vadd(x, y), reps=a.reps)
    t_dot = device_time_ms(lambda: ops.dot(x, y), reps=a.reps)
    print(f"GPU vadd: {t_add * 1e3:.1f} us ({12 * a.n / t_add / 1e6:.1f} GB/s)")
    print(f"GPU dot : {t_dot * 1e3:.1f} us ({8 * a.n / t_dot / 1e6:.1f} GB/s)", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
