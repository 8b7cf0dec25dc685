"""Timing harness shared by bench.py and the north-star CLIs.

W untimed warm-up steps, then K timed steps bracketed by barrier + device synchronise on both sides; the
elapsed time is MAX-reduced over ranks (the slowest GPU defines the job's step time)."""
from __future__ import annotations

import time

import torch

from ..parallel.dist import Context


def sync(ctx: Context) -> None:
    if ctx.device.type == "cuda":
        torch.cuda.synchronize(ctx.device)


def timed(ctx: Context, step_fn, steps: int, warmup: int) -> float:
    """Seconds for `steps` calls of step_fn (max over ranks)."""
    for _ in range(warmup):
        step_fn()
    sync(ctx)
    ctx.barrier()
    sync(ctx)
    t0 = time.perf_counter()
    for _ in range(steps):
        step_fn()
    sync(ctx)
    ctx.barrier()
    sync(ctx)
    return ctx.max_over_ranks(time.perf_counter() - t0)
