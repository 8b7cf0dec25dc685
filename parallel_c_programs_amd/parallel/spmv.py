"""Distributed CSR SpMV — north-star config "1e8-nnz power-law graph, 8 x MI355X" (ancestor: the single-core
CSR benchmark of ref 3-serial-optimization/spmv.c:170-177, 331-367).

  * partition: contiguous row blocks balanced by NNZ (not rows) — a power-law graph's heavy rows would
    otherwise pile onto one GPU. Every rank derives the same cut from the O(n) row pointer, then generates
    ONLY its own rows (bit-identical to the serial matrix), so a 1e8-nnz matrix never exists on one host.
  * iterate: y_local = A_local x (CSR-adaptive gfx950 kernel), then x <- all_gather(y) so every rank holds
    the whole vector for the next product (power-iteration pattern). The all-gather moves 4 B x n_rows per
    step over xGMI; rows blocks are padded to the largest block so it maps to one RCCL all_gather.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops.sparse import CSR, SlicedCSR, powerlaw_csr_rows, powerlaw_row_ptr, spmv
from .dist import Context


def nnz_balanced_cuts(row_ptr: torch.Tensor, parts: int) -> list[int]:
    """Row boundaries b_0=0 < ... < b_parts=n with ~equal nnz per block (binary search on row_ptr)."""
    n = row_ptr.numel() - 1
    nnz = int(row_ptr[-1])
    targets = torch.tensor([(nnz * p) // parts for p in range(1, parts)], dtype=row_ptr.dtype)
    cuts = torch.searchsorted(row_ptr, targets).tolist()
    out = [0]
    for c in cuts:
        out.append(min(max(c, out[-1]), n))
    out.append(n)
    return out


class DistributedSpMV:
    def __init__(self, ctx: Context, row_ptr: torch.Tensor, local: CSR, cuts: list[int], slices: int = 0,
                 head: float = 0.0625, balance: float = 0.0):
        self.ctx, self.cuts, self.local = ctx, cuts, local.to(ctx.device)
        self.sliced = None
        self.n = row_ptr.numel() - 1
        self.row0, self.row1 = cuts[ctx.rank], cuts[ctx.rank + 1]
        self.block = max(cuts[i + 1] - cuts[i] for i in range(ctx.world))
        if ctx.device.type == "cuda":
            if slices:  # XCD-sliced layout (ops.SlicedCSR); the plain CSR copy is then dropped
                self.sliced = SlicedCSR(self.local, slices, head, balance)
                self.local = CSR(self.local.row_ptr[-1:], self.local.col[:0], self.local.val[:0], self.local.n_cols)
            else:
                self.local.plan()
        idx = torch.cat([torch.arange(cuts[r], cuts[r + 1]) - cuts[r] + r * self.block for r in range(ctx.world)])
        self.compact = idx.to(ctx.device)
        self.gathered = torch.empty(ctx.world * self.block, dtype=torch.float32, device=ctx.device)
        self.ybuf = torch.zeros(self.block, dtype=torch.float32, device=ctx.device)

    @staticmethod
    def powerlaw(ctx: Context, n_rows: int, nnz: int, alpha: float = 2.5, seed: int = 1,
                 slices: int = 0, head: float = 0.0625, balance: float = 0.0) -> "DistributedSpMV":
        rp = powerlaw_row_ptr(n_rows, nnz, alpha, seed)
        cuts = nnz_balanced_cuts(rp, ctx.world)
        local = powerlaw_csr_rows(rp, cuts[ctx.rank], cuts[ctx.rank + 1], n_rows, seed)
        return DistributedSpMV(ctx, rp, local, cuts, slices, head, balance)

    @property
    def local_nnz(self) -> int:
        return self.sliced.nnz if self.sliced is not None else self.local.nnz

    def multiply_local(self, x: torch.Tensor) -> torch.Tensor:
        if self.sliced is not None:
            return self.sliced.spmv(x)
        return spmv(self.local, x)

    def allgather(self, y_local: torch.Tensor) -> torch.Tensor:
        if not self.ctx.distributed:
            return y_local
        self.ybuf[: y_local.numel()] = y_local
        dist.all_gather_into_tensor(self.gathered, self.ybuf)
        return self.gathered.index_select(0, self.compact)

    def step(self, x: torch.Tensor) -> torch.Tensor:
        """x (full, replicated) -> A x (full, replicated)."""
        return self.allgather(self.multiply_local(x))
