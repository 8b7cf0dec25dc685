"""Timing harness shared by bench.py and the north-star CLIs.

W untimed warm-up steps, then K timed steps bracketed by barrier + device synchronise on both sides; the
elapsed time is MAX-reduced over ranks (the slowest GPU defines the job's step time).

Per-step device time (optional): one hipEvent on the current stream at every step boundary (K + 1 events, no extra
synchronisation inside the loop), so a wall-clock outlier can be attributed: a slow step in the event times is
device work (a slow kernel or a collective waiting on a peer), wall time without it is the host (a descheduled
launch thread, a page fault) or work outside the step (ref 5-cuda-region-growing/raycast.cu:832-846 times each
phase on its own)."""
from __future__ import annotations

import statistics
import time

import torch

from ..parallel.dist import Context


def sync(ctx: Context) -> None:
    if ctx.device.type == "cuda":
        torch.cuda.synchronize(ctx.device)


def timed(ctx: Context, step_fn, steps: int, warmup: int, per_step: list | None = None) -> float:
    """Seconds for `steps` calls of step_fn (max over ranks). per_step (a list): this rank's time of each timed step
    in ms is appended — hipEvent device time on a GPU, host wall time on the CPU."""
    for _ in range(warmup):
        step_fn()
    cuda = ctx.device.type == "cuda"
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)] if per_step is not None and cuda else None
    host = [] if per_step is not None and not cuda else None
    sync(ctx)
    ctx.barrier()
    sync(ctx)
    t0 = time.perf_counter()
    if evs:
        evs[0].record()
    for i in range(steps):
        if host is not None:
            h0 = time.perf_counter()
        step_fn()
        if evs:
            evs[i + 1].record()
        if host is not None:
            host.append(1e3 * (time.perf_counter() - h0))
    sync(ctx)
    ctx.barrier()
    sync(ctx)
    elapsed = time.perf_counter() - t0
    if evs:
        per_step.extend(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    elif host is not None:
        per_step.extend(host)
    return ctx.max_over_ranks(elapsed)


def step_stats(ms: list) -> dict:
    """min / median / max of per-step times (ms); empty input -> {}."""
    if not ms:
        return {}
    return {"min": min(ms), "median": statistics.median(ms), "max": max(ms)}
