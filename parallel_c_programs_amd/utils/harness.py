"""Timing harness shared by bench.py and the north-star CLIs.

W untimed warm-up steps, then K timed steps bracketed by barrier + device synchronise on both sides; the
elapsed time is MAX-reduced over ranks (the slowest GPU defines the job's step time).

Per-step device time (optional): one hipEvent on the current stream at every step boundary (K + 1 events, no extra
synchronisation inside the loop), so a wall-clock outlier can be attributed: a slow step in the event times is
device work (a slow kernel or a collective waiting on a peer), wall time without it is the host (a descheduled
launch thread, a page fault) or work outside the step (ref 5-cuda-region-growing/raycast.cu:832-846 times each
phase on its own)."""
from __future__ import annotations

import gc
import os
import statistics
import sys
import time

import torch

from ..parallel.dist import Context


def sync(ctx: Context) -> None:
    if ctx.device.type == "cuda":
        torch.cuda.synchronize(ctx.device)


def timed(ctx: Context, step_fn, steps: int, warmup: int, per_step: list | None = None,
          host_ms: list | None = None, settle_ms: float = 0.0) -> float:
    """Seconds for `steps` calls of step_fn (max over ranks). per_step (a list): this rank's time of each timed step
    in ms is appended — hipEvent device time on a GPU, host wall time on the CPU. host_ms (a list): the host wall time
    of each step_fn call (enqueue time on a GPU): a device-time outlier without a host one is the device's (or a
    peer's), with one the host's. PCMX_TIMED_DIAG=1 also logs every cyclic-GC pass inside the loop to stderr.
    settle_ms > 0 (GPU): before the W warm-up steps, untimed steps until that much wall time has passed, so the timed
    steps run at the clock a running job sees: a VALU-bound kernel measured right after an idle set-up runs up to 12%
    slow while the shader clock ramps (profiles/r5_bench/README.md: 2.14 -> 2.26 GHz over the first 25 stencil
    launches, 2.33-2.42 in steady state)."""
    if settle_ms > 0 and ctx.device.type == "cuda":
        # the step count is agreed over the ranks (steps may hold collectives): 4 probe steps price one step, the
        # slowest rank's price sets the count
        sync(ctx)
        t0 = time.perf_counter()
        for _ in range(4):
            step_fn()
        sync(ctx)
        per = ctx.max_over_ranks((time.perf_counter() - t0) / 4)
        for _ in range(min(10_000, int(settle_ms / 1e3 / max(per, 1e-6)))):
            step_fn()
    for _ in range(warmup):
        step_fn()
    diag = os.environ.get("PCMX_TIMED_DIAG") == "1"
    gc_log = []
    if diag:  # diagnostic: every cyclic-GC pass inside the timed loop, with its host time
        t_gc = [0.0]

        def on_gc(phase, info):
            if phase == "start":
                t_gc[0] = time.perf_counter()
            else:
                gc_log.append((info.get("generation"), 1e3 * (time.perf_counter() - t_gc[0])))
    cuda = ctx.device.type == "cuda"
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)] if per_step is not None and cuda else None
    sync(ctx)
    ctx.barrier()
    sync(ctx)
    if diag:
        gc.callbacks.append(on_gc)
    t0 = time.perf_counter()
    if evs:
        evs[0].record()
    walls = []
    for i in range(steps):
        h0 = time.perf_counter()
        step_fn()
        if evs:
            evs[i + 1].record()
        walls.append(1e3 * (time.perf_counter() - h0))
    sync(ctx)
    ctx.barrier()
    sync(ctx)
    elapsed = time.perf_counter() - t0
    if diag:
        gc.callbacks.remove(on_gc)
        worst = max(range(steps), key=walls.__getitem__)
        print(f"[timed-diag] {getattr(step_fn, '__qualname__', step_fn)}: host ms per step max {walls[worst]:.3f} at "
              f"step {worst}, median {statistics.median(walls):.3f}; gc passes in the loop {gc_log}", file=sys.stderr,
              flush=True)
    if evs:
        per_step.extend(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    elif per_step is not None:
        per_step.extend(walls)
    if host_ms is not None:
        host_ms.extend(walls)
    return ctx.max_over_ranks(elapsed)


def step_stats(ms: list) -> dict:
    """min / median / max of per-step times (ms); empty input -> {}."""
    if not ms:
        return {}
    return {"min": min(ms), "median": statistics.median(ms), "max": max(ms)}
