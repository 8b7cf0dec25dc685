"""Distributed 2-D region growing on a Cartesian process grid (ref 2-mpi-region-growing/region.c, call stack
SURVEY §3.1: init_mpi :537 -> distribute_image :106 + distribute_image_halo :145 -> grow_region :493 ->
gather_region :391 -> write_image :572).

MI355X design (one process per GPU, RCCL over xGMI):
  * scatter: root cuts each rank's PADDED tile (interior + 1-cell image halo from the neighbouring tiles)
    out of the zero-padded image and sends it as ONE message — the reference's per-row sends plus its
    separate halo-distribution pass (region.c:106-353) collapse into P-1 messages.
  * local step: the gfx950 active-tile label-propagation kernel grows the tile to its LOCAL fixpoint
    (many sweeps per launch; SURVEY §7.5 hard part 2) — the reference's DFS flood fill (region.c:499-527).
  * exchange: pack 4 edges -> one grouped RCCL send/recv -> unpack (parallel/halo.py); the halo region
    cells act as seeds for the next local step (ref add_halo_to_stack :355).
  * termination: device-resident. The unpack kernel raises a "halo changed" flag on the device, the flag is
    MAX-all-reduced in place, and the host reads it once every CHECK_EVERY outer steps (ref finished() :435
    all-reduces MIN of local_finish every step). A window in which no rank's halo changed is a global fixpoint:
    a step whose halos did not change cannot grow anything, so every later step is a no-op too.
  * gather: each rank sends its interior once; root places the blocks (ref gather_region :391, B10).

Generalises the reference to any world size (B8: 1/2/4/8 ranks on a node, any image size).
Result is independent of P: the grown set is the seeds' connected component under |a-b| < threshold.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops
from ..ops.image import corner_seeds
from .dist import Context
from .halo import HaloExchanger2D
from .topology import CartTopology


CHECK_EVERY = 2  # outer steps per host read of the all-reduced "halo changed" flag


def _bcast_shape(ctx: Context, image: torch.Tensor | None) -> tuple[int, int]:
    hw = torch.tensor(list(image.shape) if ctx.is_root else [0, 0], dtype=torch.int64, device=ctx.device)
    ctx.broadcast_(hw, 0)
    return int(hw[0]), int(hw[1])


def scatter_tiles(ctx: Context, topo: CartTopology, image: torch.Tensor | None, H: int, W: int) -> torch.Tensor:
    """Root -> every rank: its (h+2, w+2) uint8 tile with the neighbouring tiles' pixels in the halo ring."""
    r0, r1, c0, c1 = topo.tile(ctx.rank, H, W)
    mine = torch.empty((r1 - r0 + 2, c1 - c0 + 2), dtype=torch.uint8, device=ctx.device)
    if ctx.is_root:
        padded = ops.pad1(image.to(ctx.device))
        reqs = []
        for r in range(topo.size):
            a0, a1, b0, b1 = topo.tile(r, H, W)
            blk = padded[a0:a1 + 2, b0:b1 + 2].contiguous()
            if r == 0:
                mine.copy_(blk)
            elif ctx._staged(blk):
                ctx.send(blk, r)
            else:
                reqs.append(dist.isend(blk, r))
        for q in reqs:
            q.wait()
    else:
        ctx.recv(mine, 0)
    return mine


def gather_tiles(ctx: Context, topo: CartTopology, interior: torch.Tensor, H: int, W: int) -> torch.Tensor | None:
    """Every rank -> root: interior blocks reassembled into (H, W) on root."""
    if not ctx.distributed:
        return interior.contiguous()
    if not ctx.is_root:
        ctx.send(interior.contiguous(), 0)
        return None
    full = torch.empty((H, W), dtype=interior.dtype, device=interior.device)
    r0, r1, c0, c1 = topo.tile(0, H, W)
    full[r0:r1, c0:c1] = interior
    for r in range(1, topo.size):
        a0, a1, b0, b1 = topo.tile(r, H, W)
        buf = torch.empty((a1 - a0, b1 - b0), dtype=interior.dtype, device=interior.device)
        ctx.recv(buf, r)
        full[a0:a1, b0:b1] = buf
    return full


def grow_distributed(ctx: Context, image: torch.Tensor | None, threshold: int = 2, seeds=None,
                     dims: tuple[int, int] | None = None, stats: dict | None = None) -> torch.Tensor | None:
    """Distributed region growing. `image` (H, W) uint8 is only needed on root; returns the (H, W) region
    bitmap on root (None elsewhere). `stats` receives outer-step / launch counts."""
    H, W = _bcast_shape(ctx, image) if ctx.distributed else tuple(image.shape)
    topo = CartTopology.create(ctx.world, dims)
    if ctx.distributed:
        img_p = scatter_tiles(ctx, topo, image, H, W)
    else:
        img_p = ops.pad1(image.to(ctx.device))
    r0, r1, c0, c1 = topo.tile(ctx.rank, H, W)
    reg_p = torch.zeros_like(img_p)
    for x, y in (corner_seeds(H, W) if seeds is None else seeds):
        if r0 <= y < r1 and c0 <= x < c1:
            reg_p[y - r0 + 1, x - c0 + 1] = 1
    ex = HaloExchanger2D(ctx, topo)
    outer, launches, reads = 0, 0, 0
    changed = torch.zeros(1, dtype=torch.int32, device=ctx.device)
    while True:
        launches += ops.region2d_grow_padded_(reg_p, img_p, threshold)
        outer += 1
        if not ctx.distributed:
            break
        ex.exchange_(reg_p, changed)
        if outer % CHECK_EVERY:
            continue
        ctx.all_reduce_(changed, "max")
        reads += 1
        if int(changed.item()) == 0:  # the loop's only host read-back
            break
        changed.zero_()
    if stats is not None:
        stats.update(outer_steps=outer, launches=launches, dims=topo.dims, host_reads=reads)
    return gather_tiles(ctx, topo, reg_p[1:-1, 1:-1], H, W)
