"""Nearest-neighbour halo exchange for 2-D tiles (ref 2-mpi-region-growing/region.c:145-353:
distribute_image_halo + exchange).

MI355X design: one pack kernel gathers the 4 interior edges into a contiguous buffer, the 4 sends and
4 receives go out as ONE grouped RCCL operation (Context.neighbour_exchange: a list all_to_all ->
ncclGroupStart/End, point-to-point over xGMI), then one unpack kernel fills the halo ring. The grouped call is deadlock-free by
construction, replacing the reference's parity-ordered blocking Send/Recv (which relied on eager buffering,
B9). Absent neighbours (grid edge) are skipped and their halo is left untouched.
"""
from __future__ import annotations

import torch

from ..ops.halo import BOTTOM, LEFT, RIGHT, TOP, edge_slices, pack_edges, unpack_halo_
from .dist import Context
from .topology import CartTopology


class HaloExchanger2D:
    """Exchanges the 1-cell halo ring of a padded (H+2, W+2) tile with the N/S/W/E neighbours."""

    def __init__(self, ctx: Context, topo: CartTopology):
        self.ctx, self.topo = ctx, topo
        self.nb = topo.neighbours(ctx.rank)

    def mask(self) -> int:
        m = 0
        m |= TOP if self.nb["north"] >= 0 else 0
        m |= BOTTOM if self.nb["south"] >= 0 else 0
        m |= LEFT if self.nb["west"] >= 0 else 0
        m |= RIGHT if self.nb["east"] >= 0 else 0
        return m

    def exchange_(self, tile: torch.Tensor, changed: torch.Tensor | None = None) -> torch.Tensor:
        """In-place halo update of `tile`; returns the received edge buffer. `changed` (int32 [1]) is raised to 1
        on the device when any halo cell takes a new value."""
        H, W = tile.shape[0] - 2, tile.shape[1] - 2
        send = pack_edges(tile)
        recv = torch.zeros_like(send)
        if not self.ctx.distributed:
            return recv
        top, bottom, left, right = edge_slices(H, W)
        # my top edge -> north neighbour's bottom halo; north's bottom edge -> my top halo, etc.
        pairs, recv_parts = [], []
        for side, sl in (("north", top), ("south", bottom), ("west", left), ("east", right)):
            peer = self.nb[side]
            if peer < 0:
                continue
            buf = torch.empty_like(send[sl])
            recv_parts.append((buf, sl))
            pairs.append((peer, send[sl].contiguous(), buf))
        self.ctx.neighbour_exchange(pairs)  # ONE RCCL call for the up-to-4 neighbours (Context.neighbour_exchange)
        for buf, sl in recv_parts:
            recv[sl] = buf
        unpack_halo_(tile, recv, self.mask(), changed)
        return recv
