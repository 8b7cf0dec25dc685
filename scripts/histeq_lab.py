"""Histogram-equalisation lab: GPU paths vs the serial host reference (bit-exact) and per-call timing.

usage: python scripts/histeq_lab.py   (one GPU)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parallel_c_programs_amd import ops  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    for side, hi in ((512, 200), (512, 3), (2048, 256), (4096, 200), (4096, 2), (8192, 256)):
        img = torch.randint(0, hi, (side, side), dtype=torch.uint8, generator=g)
        ref = ops.histeq(img, "serial")
        gi = img.to(dev)
        for method in ("auto", "multiblock"):
            out = ops.histeq(gi, method).cpu()
            ok = torch.equal(out, ref)
            us = timeit(lambda: ops.histeq(gi, method))
            gbps = 2 * img.numel() / us / 1e3
            print(f"side {side:5d} values<{hi:3d} {method:10s} exact={ok} {us:8.1f} us  {img.numel() / us / 1e3:7.1f} Gpix/s "
                  f"({gbps:6.0f} GB/s img+out)", flush=True)
            assert ok


if __name__ == "__main__":
    main()
