"""Halo pack/unpack for padded 2-D tiles (replaces the reference's MPI derived datatypes,
2-mpi-region-growing/region.c:86-102). One launch gathers the four interior edges into a contiguous
buffer [top W | bottom W | left H | right H]; one launch scatters a received buffer into the halo ring."""
from __future__ import annotations

import torch

from .._native import ops

TOP, BOTTOM, LEFT, RIGHT = 1, 2, 4, 8


def pack_edges(tile: torch.Tensor) -> torch.Tensor:
    if tile.is_cuda:
        return ops().pack_edges(tile)
    return torch.cat([tile[1, 1:-1], tile[-2, 1:-1], tile[1:-1, 1], tile[1:-1, -2]]).contiguous()


def unpack_halo_(tile: torch.Tensor, buf: torch.Tensor, mask: int = TOP | BOTTOM | LEFT | RIGHT,
                 changed: torch.Tensor | None = None) -> torch.Tensor:
    """Scatter `buf` into the halo ring; `changed` (int32 [1], same device) is set to 1 when any halo cell takes a
    new value (device-resident change detection: nothing is read back to the host)."""
    if tile.is_cuda:
        ops().unpack_halo_(tile, buf, int(mask), changed)
        return tile
    H, W = tile.shape[0] - 2, tile.shape[1] - 2
    parts = []
    if mask & TOP:
        parts.append((tile[0, 1:-1], buf[:W]))
    if mask & BOTTOM:
        parts.append((tile[-1, 1:-1], buf[W:2 * W]))
    if mask & LEFT:
        parts.append((tile[1:-1, 0], buf[2 * W:2 * W + H]))
    if mask & RIGHT:
        parts.append((tile[1:-1, -1], buf[2 * W + H:]))
    for dst, src in parts:
        if changed is not None and not torch.equal(dst, src):
            changed.fill_(1)
        dst.copy_(src)
    return tile


def edge_slices(H: int, W: int):
    """Slices of the packed buffer: top, bottom, left, right."""
    return slice(0, W), slice(W, 2 * W), slice(2 * W, 2 * W + H), slice(2 * W + H, 2 * W + 2 * H)
