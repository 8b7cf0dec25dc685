"""Timers with the reference's output format (print_time, ref 3-serial-optimization/spmv.c:164-168:
"Time : %f s") plus HIP-event device timing."""
from __future__ import annotations

import contextlib
import time

import torch


def print_time(seconds: float) -> None:
    print(f"Time : {seconds:f} s", flush=True)


@contextlib.contextmanager
def wall_timer(label: str | None = None, sync_device: bool = True, out: dict | None = None):
    """Wall-clock region (device-synchronised on both sides when a GPU is in use)."""
    if sync_device and torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    yield
    if sync_device and torch.cuda.is_available():
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if out is not None:
        out[label or "t"] = dt
    if label is not None:
        print(label, flush=True)
        print_time(dt)


def device_time_ms(fn, reps: int = 10, warmup: int = 2) -> float:
    """Median of `reps` HIP-event-timed calls of fn()."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]
