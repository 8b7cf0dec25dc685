"""Distributed CSR SpMV — north-star config "1e8-nnz power-law graph, 8 x MI355X" (ancestor: the single-core
CSR benchmark of ref 3-serial-optimization/spmv.c:170-177, 331-367).

  * partition: contiguous row blocks balanced by NNZ (not rows) — a power-law graph's heavy rows would
    otherwise pile onto one GPU. Every rank derives the same cut from the O(n) row pointer, then generates
    ONLY its own rows (bit-identical to the serial matrix), so a 1e8-nnz matrix never exists on one host.
  * iterate (power-iteration pattern): y_local = A_local x, then every rank needs all of y as the next x.
  * padded vector layout: each rank's row block is cut into `chunks` pieces of L rows (the block padded to
    chunks x L); vector entry of global row g (rank r, local row l) lives at
        p(g) = (l // L) * (world * L) + r * L + (l % L).
    Chunk c of every rank is then ONE contiguous all_gather_into_tensor region, so RCCL writes the
    gathered y straight into the next x: no staging copy, no index_select. The matrix's column indices are
    renumbered into this layout once at set-up (on one rank the layout is the identity).
  * overlap: the product runs chunk by chunk; chunk c's all-gather is issued (async, RCCL's own stream
    waits only for chunk c's kernel) while chunk c+1 is multiplied, so only the last chunk's gather is
    exposed: t_step ~= t_local + t_gather / chunks when t_gather <= t_local (docs/ARCHITECTURE.md, SpMV).
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


def padded_index(cuts: list[int], chunks: int, L: int, device="cpu") -> torch.Tensor:
    """p(g) of every global row/column g (int64 [n]) for the padded layout described above."""
    n, W = cuts[-1], len(cuts) - 1
    g = torch.arange(n, device=device)
    ends = torch.tensor(cuts[1:], device=device)
    owner = torch.searchsorted(ends, g, right=True)
    local = g - torch.tensor(cuts, device=device)[owner]
    return (local // L) * (W * L) + owner * L + local % L


class DistributedSpMV:
    def __init__(self, ctx: Context, row_ptr: torch.Tensor, local: CSR, cuts: list[int], slices: int = 0,
                 head: float = 0.0625, balance: float = 0.0, chunks: int | None = None, item_nnz: int = 1024):
        W, dev = ctx.world, ctx.device
        self.ctx, self.cuts = ctx, cuts
        self.n = row_ptr.numel() - 1
        self.row0, self.row1 = cuts[ctx.rank], cuts[ctx.rank + 1]
        self.rows = self.row1 - self.row0
        self.block = max(1, max(cuts[i + 1] - cuts[i] for i in range(W)))
        C = chunks if chunks else (1 if W == 1 else 4)
        C = max(1, min(int(C), self.block))
        self.chunks = C
        self.L = -(-self.block // C)
        self.n_pad = C * W * self.L
        self.colmap = padded_index(cuts, C, self.L, dev)  # identity when W == 1
        col = local.col.to(dev)
        if W > 1:
            col = self.colmap[col.long()].to(torch.int32)
        m = CSR(local.row_ptr.to(dev), col, local.val.to(dev), self.n_pad)
        self.sliced = bool(slices) and dev.type == "cuda"
        self.parts = []  # (first local row, last local row + 1, CSR or SlicedCSR)
        for c in range(C):
            a, b = min(c * self.L, self.rows), min((c + 1) * self.L, self.rows)
            part = m.row_block(a, b)
            if dev.type == "cuda":
                part = SlicedCSR(part, slices, head, balance, item_nnz) if self.sliced else part.plan()
            self.parts.append((a, b, part))
        del m, col
        self.send = torch.zeros(C, self.L, dtype=torch.float32, device=dev)  # tails of short chunks stay 0
        self.bufs = [torch.zeros(self.n_pad, dtype=torch.float32, device=dev) for _ in range(2)]

    @staticmethod
    def powerlaw(ctx: Context, n_rows: int, nnz: int, alpha: float = 2.5, seed: int = 1,
                 slices: int = 0, head: float = 0.0625, balance: float = 0.0,
                 chunks: int | None = None, item_nnz: int = 1024) -> "DistributedSpMV":
        rp = powerlaw_row_ptr(n_rows, nnz, alpha, seed)
        cuts = nnz_balanced_cuts(rp, ctx.world)
        local = powerlaw_csr_rows(rp, cuts[ctx.rank], cuts[ctx.rank + 1], n_rows, seed)
        return DistributedSpMV(ctx, rp, local, cuts, slices, head, balance, chunks, item_nnz)

    @property
    def local_nnz(self) -> int:
        return sum(p.nnz for _, _, p in self.parts)

    # ---- layout conversion (natural global order <-> padded layout)
    def to_padded(self, x: torch.Tensor) -> torch.Tensor:
        xp = torch.zeros(self.n_pad, dtype=torch.float32, device=self.ctx.device)
        xp[self.colmap] = x.to(xp.device, torch.float32)
        return xp

    def from_padded(self, xp: torch.Tensor) -> torch.Tensor:
        return xp[self.colmap]

    def local_positions(self) -> torch.Tensor:
        """Padded positions of this rank's rows, in local row order."""
        return self.colmap[self.row0:self.row1]

    # ---- products
    def _mul(self, part, xp: torch.Tensor, dst: torch.Tensor) -> None:
        if self.sliced:
            part.spmv(xp, dst)
        else:
            dst.copy_(spmv(part, xp))

    def step_padded(self, xp: torch.Tensor) -> torch.Tensor:
        """xp (padded layout, replicated) -> A xp (padded layout, replicated on every rank). The result lives in
        one of two internal buffers; the buffer that is not `xp` is overwritten."""
        out = self.bufs[0] if xp.data_ptr() != self.bufs[0].data_ptr() else self.bufs[1]
        W, L = self.ctx.world, self.L
        if not self.ctx.distributed:
            for c, (a, b, part) in enumerate(self.parts):
                self._mul(part, xp, out[c * L:c * L + (b - a)])
            return out
        works = []
        for c, (a, b, part) in enumerate(self.parts):
            if b > a:
                self._mul(part, xp, self.send[c, :b - a])
            works.append(dist.all_gather_into_tensor(out[c * W * L:(c + 1) * W * L], self.send[c], async_op=True))
        for w in works:
            w.wait()
        return out

    def step(self, x: torch.Tensor) -> torch.Tensor:
        """x (full, natural order, replicated) -> A x (full, natural order, replicated)."""
        return self.from_padded(self.step_padded(self.to_padded(x)))

    def reference_local(self, xp: torch.Tensor) -> torch.Tensor:
        """fp64 product of this rank's rows with xp (padded layout), in local row order."""
        outs = []
        for a, b, part in self.parts:
            if isinstance(part, SlicedCSR):
                outs.append(part.reference(xp))
            else:
                rows = torch.repeat_interleave(torch.arange(part.n_rows, device=xp.device),
                                               (part.row_ptr[1:] - part.row_ptr[:-1]).to(xp.device))
                y = torch.zeros(part.n_rows, dtype=torch.float64, device=xp.device)
                y.index_add_(0, rows, part.val.double().to(xp.device) * xp.double()[part.col.long().to(xp.device)])
                outs.append(y)
        return torch.cat(outs) if outs else torch.zeros(0, dtype=torch.float64, device=xp.device)
