"""MALL (Infinity Cache) lab: does a second streaming pass over the same array run above the HBM rate, i.e. do
the reduce kernel's (non-temporal) loads leave the data in the 256-MB memory-side cache? Times ops.reduce and
torch.sum over arrays of 32 MB .. 1 GB, each pass directly after another pass over the same array, and after a
pass over a different 1-GB array (cold). Run: python scripts/mall_lab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402


def t(fn, pre, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot = 0.0
    for _ in range(reps):
        pre()
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        tot += e0.elapsed_time(e1)
    return tot / reps


dev = torch.device("cuda", 0)
flush = torch.empty(1 << 28, device=dev).fill_(1.0)  # 1 GB
for mb in (32, 64, 128, 192, 256, 384, 512, 1024):
    x = torch.rand(mb << 18, device=dev)
    for name, fn in (("ops.reduce", lambda: ops.reduce(x, "sum")), ("torch.sum", lambda: x.sum())):
        warm = t(fn, fn)
        cold = t(fn, lambda: ops.reduce(flush, "sum"))
        print(f"{mb:5d} MB {name:10s} after same-array pass {warm:.4f} ms ({mb / 1024 / warm:.2f} TB/s)  "
              f"after 1-GB other pass {cold:.4f} ms ({mb / 1024 / cold:.2f} TB/s)", flush=True)
    del x
