"""Distributed reductions and scans over RCCL — the north-star "global reduction + prefix-scan 1e9 f32
across 8 x MI355X" (ancestors: MPI_Allreduce, ref 2-mpi-region-growing/region.c:435-440; the histogram CDF,
ref 4-histogram-equalization-openmp-pthreads/histogram_serial.c:29-34).

Design for xGMI (7 point-to-point links per GPU, ring collectives are per-link bound):
  * global_reduce: reduce locally at HBM speed first (gfx950 kernel, ~7 TB/s), then all-reduce ONE scalar —
    the collective is latency-bound (tens of µs), never a 4 GB transfer.
  * global_scan: reduce-then-scan. Local totals (one f32 per rank) are all-gathered, each rank forms its
    exclusive offset on the device and feeds it to the single-pass scan kernel as its initial value: the
    array is read twice and written once (3 x 4 B/element), no fix-up pass.
  * allreduce_buckets: large-vector all-reduce in fixed-size buckets (default 64 MiB) so a bucket pipeline
    keeps every link busy and no single giant message monopolises RCCL's buffers.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops
from .dist import Context


def global_reduce(x: torch.Tensor, ctx: Context, op: str = "sum") -> torch.Tensor:
    """op over the concatenation of every rank's x (0-d tensor, identical on every rank)."""
    local = ops.reduce(x, op)
    if x.dtype == torch.float32 and op == "sum":
        local = local.double() if not x.is_cuda else local
    t = local.reshape(1).clone()
    ctx.all_reduce_(t, op)
    return t.reshape(())


def global_scan(x: torch.Tensor, ctx: Context, exclusive: bool = False, comm: bool = True) -> torch.Tensor:
    """Prefix sum of the rank-ordered concatenation of every rank's x; returns this rank's slice.

    One rank: the single-pass look-back scan alone (8 B/element of HBM traffic). Several ranks: a local
    HBM-bound reduce (4 B/element), an all-gather of the per-rank totals over RCCL, and the scan seeded
    with the sum of the lower ranks' totals (12 B/element, no second fix-up pass over the output).
    comm=False (bench attribution only): the same kernels with the all-gather skipped (every rank's offset then
    comes from its own total alone: NOT the global scan)."""
    if not ctx.distributed:
        return ops.scan(x, exclusive=exclusive)
    total = ops.reduce(x, "sum").reshape(1).float()
    totals = torch.empty(ctx.world, dtype=torch.float32, device=x.device)
    if comm:
        dist.all_gather_into_tensor(totals, total)  # one collective into one tensor, no per-rank list
    else:
        totals.copy_(total.expand(ctx.world))
    before = totals[:ctx.rank].sum().reshape(1) if ctx.rank else torch.zeros(1, dtype=torch.float32, device=x.device)
    return ops.scan(x, exclusive=exclusive, init=before)


def allreduce_buckets(t: torch.Tensor, ctx: Context, bucket_bytes: int = 64 << 20, op: str = "sum") -> torch.Tensor:
    """In-place bucketed all-reduce of a contiguous tensor."""
    if not ctx.distributed:
        return t
    flat = t.view(-1)
    per = max(1, bucket_bytes // flat.element_size())
    works = []
    for s in range(0, flat.numel(), per):
        works.append(dist.all_reduce(flat[s:s + per], op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                                                            "min": dist.ReduceOp.MIN}[op], async_op=True))
    for w in works:
        w.wait()
    return t


def scatter_rows(full: torch.Tensor | None, ctx: Context, counts: list[int], shape_tail: tuple, dtype,
                 device) -> torch.Tensor:
    """Root scatters consecutive row blocks of `full` (counts[r] rows to rank r): ONE message per rank
    (ref distribute_image sends one message per row per rank, region.c:106-143)."""
    mine = torch.empty((counts[ctx.rank], *shape_tail), dtype=dtype, device=device)
    if not ctx.distributed:
        mine.copy_(full)
        return mine
    if ctx.is_root:
        start = 0
        reqs = []
        for r, n in enumerate(counts):
            blk = full[start:start + n].contiguous()
            start += n
            if r == 0:
                mine.copy_(blk)
            else:
                reqs.append(dist.isend(blk, r))
        for q in reqs:
            q.wait()
    else:
        dist.recv(mine, 0)
    return mine


def gather_rows(mine: torch.Tensor, ctx: Context, counts: list[int]) -> torch.Tensor | None:
    """Inverse of scatter_rows: root receives every rank's row block (one message per rank)."""
    if not ctx.distributed:
        return mine.clone()
    if ctx.is_root:
        parts = [mine]
        for r in range(1, ctx.world):
            buf = torch.empty((counts[r], *mine.shape[1:]), dtype=mine.dtype, device=mine.device)
            dist.recv(buf, r)
            parts.append(buf)
        return torch.cat(parts)
    dist.send(mine.contiguous(), 0)
    return None
