"""Reduce/scan rank lab: one rank's device work per step of the strong-scaled "1e9 f32 across N GPUs" reduce and
scan (1e9 / N elements per rank) on one GPU, without the collectives:

  reduce   local HBM reduce (what precedes the one-scalar RCCL all-reduce)
  scan     local reduce + scan seeded with a device offset (what global_scan runs around its all-gather of totals)
  scan1    the plain single-rank scan (N = 1 path, 8 B/element)

Prints ms and GB/s (4 B/element for reduce, 8 B/element for the scans, as bench.py counts them), i.e. the
compute-side bound of each N's step before the collective latency. Run: python scripts/collective_rank_lab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    total = 10 ** 9
    for world in (1, 2, 4, 8):
        n = -(-total // world)
        x = torch.empty(n, device=dev)
        ops.rand_uniform_(x, 3000, 0.0, 1.0)
        off = torch.full((1,), 123.0, device=dev)
        t_red = timed(lambda: ops.reduce(x, "sum"))
        t_scan = timed(lambda: ops.scan(x, init=ops.reduce(x, "sum").reshape(1).float() * 0 + off))
        t_scan1 = timed(lambda: ops.scan(x))
        print(f"N={world} per-rank {n:11d}  reduce {t_red:.4f} ms {4 * n / t_red / 1e6:6.0f} GB/s   "
              f"scan(reduce+seeded) {t_scan:.4f} ms {8 * n / t_scan / 1e6:6.0f} GB/s   "
              f"scan1 {t_scan1:.4f} ms {8 * n / t_scan1 / 1e6:6.0f} GB/s", flush=True)
        del x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
