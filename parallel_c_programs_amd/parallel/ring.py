"""Token chain over point-to-point messages (ref 1-introduction/mpi.c:5-44, call stack SURVEY §3.6).

The token travels up from rank 0 to rank P-1 (each hop +1) and back down (each hop +1), so rank 0 ends
with 2P-2. Printed lines keep the reference's text ("Rank %d received %d \\n" / "Rank %d sent %d \\n").
Over RCCL the token is a 1-element int32 device tensor (a latency probe of the xGMI path).
"""
from __future__ import annotations

import sys

import torch
import torch.distributed as dist

from .dist import Context


def _say(msg: str, out) -> None:
    out.write(msg)
    out.flush()


def token_ring(ctx: Context, out=None, verbose: bool = True) -> int:
    out = sys.stdout if out is None else out
    rank, size = ctx.rank, ctx.world
    msg = torch.zeros(1, dtype=torch.int32, device=ctx.device)
    if rank != 0:
        dist.recv(msg, rank - 1)
        if verbose:
            _say(f"Rank {rank} received {int(msg.item())} \n", out)
        msg += 1
    if rank < size - 1:
        dist.send(msg, rank + 1)
        if verbose:
            _say(f"Rank {rank} sent {int(msg.item())} \n", out)
        dist.recv(msg, rank + 1)
        if verbose:
            _say(f"Rank {rank} received {int(msg.item())} \n", out)
        msg += 1
    if rank != 0:
        dist.send(msg, rank - 1)
        if verbose:
            _say(f"Rank {rank} sent {int(msg.item())} \n", out)
    return int(msg.item())
