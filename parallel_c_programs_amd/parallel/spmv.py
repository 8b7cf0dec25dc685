"""Distributed CSR SpMV — north-star config "1e8-nnz power-law graph, 8 x MI355X" (ancestor: the single-core
CSR benchmark of ref 3-serial-optimization/spmv.c:170-177, 331-367).

  * partition: contiguous row blocks balanced by NNZ (not rows) — a power-law graph's heavy rows would
    otherwise pile onto one GPU. Every rank derives the same cut from the O(n) row pointer, then generates
    ONLY its own rows (bit-identical to the serial matrix), so a 1e8-nnz matrix never exists on one host.
  * iterate (power-iteration pattern): y_local = A_local x, then every rank needs the entries of y its rows
    reference as the next x. Each rank's row block is cut into `chunks` pieces of L rows.
  * exchange="ghost" (default at N > 1): each rank keeps only the x entries its nonzeros reference — its own
    rows plus "ghost" entries owned by other ranks (63% of the 1e7 columns per rank at N=8 on the 1e8-nnz graph)
    — in a compact local vector laid out chunk-major, owner-minor:
        [chunk 0: ghosts of ranks 0..W-1 except r, in rank order | own rows of chunk 0] [chunk 1: ...] ...
    so one chunk's product is one contiguous own segment and its ghosts one contiguous region: after chunk c's
    product, its send entries (one index list per peer, fixed at set-up) are packed and moved by ONE
    collective (Context.exchange: RCCL grouped per-peer sends over the point-to-point xGMI links, no all-gather of the
    whole y) straight into the peers' ghost regions, while chunk c+1 is multiplied. The column indices are renumbered
    into this layout once at set-up; on one rank it is the identity.
  * exchange="allgather": the padded replicated layout (every rank holds all of y): entry of global row g
    (rank r, local row l) lives at p(g) = (l // L) * (world * L) + r * L + (l % L), so chunk c of every rank is
    ONE contiguous all_gather_into_tensor region written straight into the next x.
  * overlap (both): chunk c's exchange is issued async (RCCL's own stream waits only for chunk c's kernel)
    while chunk c+1 is multiplied, so only the last chunk's exchange is exposed (docs/ARCHITECTURE.md, SpMV).
  * column split (ghost layout, 2 chunks, N > 1; round 4): every product is also cut at the first layout column of
    chunk 1, and a step multiplies the chunk-0 columns of both row chunks first, waits for the previous step's
    chunk-1 exchange only then, and leaves its own chunk-1 exchange in flight for the next step: in steady state no
    exchange is exposed, at the cost of 4 product launches per step instead of 2 (_step_colsplit).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops.sparse import CSR, PackedLayoutUnavailable, SlicedCSR, powerlaw_csr_rows, powerlaw_row_ptr, spmv
from ..ops.vector import gather_
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


def auto_slices(n_cols: int) -> int:
    """XCD slices for a vector of n_cols entries: about 400K columns (1.6 MB of x) per slice, a multiple of 8 in
    [8, 32]. Measured (one MI355X, 1e8-nnz power-law): 1e7 columns 16/24/32 slices = 0.711/0.675/0.688 ms per
    product (after predication; 16 was best before it); one N=8 rank's 6.4M-column ghost layout 16/24/32 =
    0.120/0.125/0.128 ms (profiles/r2_spmv/rank_lab.txt, slices_sweep.txt)."""
    return int(min(32, max(8, 8 * round(n_cols / 400_000 / 8))))


class ColSplitCSR:
    """A row block split at layout column B into the CSR of its columns < B and of the rest (the column-split schedule
    on the plain CSR path: CPU / gloo tests and GPUs without slices): product_phase(x, 0) multiplies the first,
    product_phase(x, 1, dst) adds the second (same fp32 sum on every path: (A0 x) + (A1 x))."""

    def __init__(self, m: CSR, B: int):
        self.n_rows, self.nnz = m.n_rows, m.nnz
        self.parts = []
        rows = torch.repeat_interleave(torch.arange(m.n_rows, device=m.col.device), m.row_ptr[1:] - m.row_ptr[:-1])
        for keep in (m.col < B, m.col >= B):
            cnt = torch.bincount(rows[keep], minlength=m.n_rows)
            rp = torch.zeros(m.n_rows + 1, dtype=torch.int64, device=m.col.device)
            rp[1:] = cnt.cumsum(0)
            part = CSR(rp, m.col[keep].contiguous(), m.val[keep].contiguous(), m.n_cols)
            self.parts.append(part.plan() if part.val.is_cuda else part)
        self.tmp = {}

    def product_phase(self, x: torch.Tensor, phase: int, key=0, dst: torch.Tensor | None = None) -> None:
        if phase == 0:
            self.tmp[key] = spmv(self.parts[0], x)
        else:
            dst.copy_(self.tmp.pop(key) + spmv(self.parts[1], x))

    def product(self, x: torch.Tensor) -> torch.Tensor:
        return spmv(self.parts[0], x) + spmv(self.parts[1], x)

    def reference(self, x: torch.Tensor) -> torch.Tensor:
        y = torch.zeros(self.n_rows, dtype=torch.float64, device=x.device)
        for p in self.parts:
            rows = torch.repeat_interleave(torch.arange(p.n_rows, device=x.device), (p.row_ptr[1:] - p.row_ptr[:-1]).to(x.device))
            y.index_add_(0, rows, p.val.double().to(x.device) * x.double()[p.col.long().to(x.device)])
        return y


def _sliced_product_phase(self: SlicedCSR, x: torch.Tensor, phase: int, key=0, dst: torch.Tensor | None = None,
                          send: tuple | None = None) -> None:
    """Column-split product of a SlicedCSR: phase 0 = the products of the slices below the split (partials only),
    phase 1 = the products of the others, then the combine + fix-up (+ the send-buffer pack, `send`) into dst."""
    half = self.n_slices // 16
    blocks = self.phase_blocks[phase] << 8  # resident product blocks per CU of this phase's launch (0: the default)
    if phase == 0:
        self.spmv(x, mode=16 | blocks, phases=(0, half))
    else:
        self.spmv(x, mode=16 | blocks, phases=(half, half))
        self.spmv(x, dst, mode=32, send=send)


SlicedCSR.product_phase = _sliced_product_phase


class DistributedSpMV:
    def __init__(self, ctx: Context, row_ptr: torch.Tensor, local: CSR, cuts: list[int], slices: int = 0,
                 head: float = 0.0625, balance: float = 0.0, chunks: int | None = None, item_nnz: int = 0,
                 exchange: str = "ghost", keep_plain: bool = False, colsplit: bool | None = None,
                 chunk0_frac: float | None = None):
        W, dev = ctx.world, ctx.device
        if exchange not in ("ghost", "allgather"):
            raise ValueError("exchange: 'ghost' or 'allgather'")
        self.ctx, self.cuts, self.exchange = ctx, cuts, exchange if W > 1 else "ghost"
        self.n = row_ptr.numel() - 1
        self.row0, self.row1 = cuts[ctx.rank], cuts[ctx.rank + 1]
        self.rows = self.row1 - self.row0
        self.block = max(1, max(cuts[i + 1] - cuts[i] for i in range(W)))
        # defaults from one rank's products at N=8 (scripts/spmv_rank_lab.py, profiles/r2_spmv/rank_lab.txt): every
        # chunk is a kernel + combine launch pair over 1/C of a small matrix (4 chunks 0.161 ms, 2: 0.134, 1: 0.113),
        # so 2 chunks balance the exposed last-chunk exchange against the launch overhead; 512-nnz items give the
        # smaller per-rank matrices more waves (2 chunks: 0.134 -> 0.127 ms)
        C = chunks if chunks else (1 if W == 1 else 2)
        # round 5: a rank of <= 16M nonzeros (N = 8 on the 1e8 matrix) takes 384-nnz items (6 per lane): its short
        # phase launches give each wave only ~2 items, and 384 fills the tail better than 512 (step 0.1163-0.1168 ->
        # 0.1149 ms with 2 resident blocks per slice in the paired launch; N = 4 indifferent, 256: slower;
        # profiles/r5_spmv/items_384_ab.txt)
        auto_items = not item_nnz
        local_nnz = int(local.row_ptr[-1] - local.row_ptr[0])
        item_nnz = item_nnz or (1024 if W == 1 else 384 if local_nnz <= 16_000_000 else 512)
        C = max(1, min(int(C), self.block))
        self.chunks = C
        self.L = -(-self.block // C)
        # row chunk boundaries in local-row space, the same on every rank (cb[c] <= local row < cb[c + 1]: chunk c).
        # Uniform (c * L) except the 2-chunk ghost layout of a distributed GPU step, whose chunk 0 takes a fraction
        # chunk0_frac of the rows (round 6, default CHUNK0_FRAC): the column-split step posts chunk 0's exchange after
        # chunk 0's combine and needs it at the top of the next step, so its window is chunk 1's phase-1 products +
        # combine, while chunk 1's window is the fixed paired phase-0 launch. A smaller chunk 0 both shrinks chunk 0's
        # exchange and widens its window (docs/ARCHITECTURE.md, SpMV exchange model; profiles/r6_spmv/).
        if chunk0_frac is None:
            chunk0_frac = self.CHUNK0_FRAC if (C == 2 and self.exchange == "ghost" and ctx.distributed and slices
                                               and dev.type == "cuda" and colsplit is not False) else 0.5
        if C == 2 and self.exchange == "ghost" and chunk0_frac != 0.5:
            L0 = max(1, min(self.block - 1, int(round(float(chunk0_frac) * self.block))))
            self.cb = [0, L0, max(self.block, L0)]
        else:
            self.cb = [c * self.L for c in range(C + 1)]
        self.cb[-1] = max(self.cb[-1], self.block)
        self.chunk0_frac = self.cb[1] / max(1, self.block) if C > 1 else 1.0
        col = local.col.to(dev)
        if self.exchange == "allgather":
            self.n_pad = C * W * self.L
            self.colmap = padded_index(cuts, C, self.L, dev)  # identity when W == 1
            if W > 1:
                col = self.colmap[col.long()].to(torch.int32)
        else:
            col = self._ghost_layout(col)
        m = CSR(local.row_ptr.to(dev), col, local.val.to(dev), self.n_pad)
        # keep_plain: the rank's rows as one plain CSR in layout columns (the vendor-library baseline: torch sparse
        # CSR x dense vector = hipSPARSE on ROCm)
        self.plain = m if keep_plain else None
        if slices < 0:
            slices = auto_slices(self.n_pad)
        # column split (2 chunks, ghost layout, N > 1): every product is cut at B = the first layout column of chunk
        # 1, so the next step multiplies the chunk-0 columns (their exchange overlapped this step's chunk-1 product)
        # while the chunk-1 exchange is still in flight, and only then the chunk-1 columns (see step_padded)
        B = self.ghost0[1] if self.exchange == "ghost" and C == 2 else 0
        if colsplit is None:
            # default only where it pays: the sliced GPU product (its phase launches split the same slice partials, so
            # the combined row sums do not change order). On the plain CSR path (CPU / gloo) (A0 x) + (A1 x) would only
            # change the fp32 summation order, so it is opt-in there (ColSplitCSR, tests)
            colsplit = ctx.distributed and 0 < B < self.n_pad and bool(slices) and dev.type == "cuda"
        self.colsplit = bool(colsplit) and 0 < B < self.n_pad
        self.col_split = B if self.colsplit else 0
        if self.colsplit and slices:
            slices = max(16, 16 * round(slices / 16))  # 8-slice phases on each side of the split
        self.slices = slices
        self.sliced = bool(slices) and dev.type == "cuda"
        self.parts = []  # (first local row, last local row + 1, CSR, SlicedCSR or ColSplitCSR)
        for c in range(C):
            a, b = self.chunk_rows(c)
            part = m.row_block(a, b)
            if self.sliced:
                try:
                    sc = SlicedCSR(part, slices, head, balance, item_nnz, col_split=self.col_split)
                except PackedLayoutUnavailable:  # 384-nnz items need the packed index stream: an automatic choice
                    if not (auto_items and item_nnz == 384):  # falls back to 512
                        raise
                    item_nnz = 512
                    sc = SlicedCSR(part, slices, head, balance, item_nnz, col_split=self.col_split)
                part = sc
                # one rank: the in-library combine + fix-up (two launches, 69 + 5 us on the 1e8-nnz matrix) beats the
                # fused combine (77 us: its waves holding split rows sum their runs serially); distributed steps fuse
                # (fewer launches on 1/N of the rows, and the send-buffer pack rides along): profiles/r5_spmv/
                part.fused_combine = ctx.distributed
                # the paired phase-0 launch (two matrices, two slices per XCD) of a small rank: 1 resident block per
                # slice and CU instead of 3 — N = 8 0.1182 -> 0.1161 ms per step, N = 4 0.2026 -> 0.2005, N = 2 0.3932 ->
                # 0.3951 (kept at 3 there); with 384-nnz items 2 (0.1149 against 0.1153-0.1156 at 1); phase 1
                # indifferent (profiles/r5_spmv/phase_blocks_sweep.txt, items_384_ab.txt)
                part.phase_blocks = (2, 0) if item_nnz == 384 else (1, 0) if W >= 4 else (0, 0)
            elif self.colsplit:
                part = ColSplitCSR(part, self.col_split)
            elif dev.type == "cuda":
                part = part.plan()
            self.parts.append((a, b, part))
        self._pending = [[], []]  # column split: the exchange works of the previous step's chunks 0 and 1
        self.comm = True  # False (bench attribution only): every exchange skipped, the same kernels run
        self._segs = [None] * C  # per chunk: the exchange's (send offsets, counts, recv offsets, counts), built once
        # the send-buffer pack in the sliced product's combine epilogue (False: a separate gather pass, the round-4 form)
        self.fuse_pack = True
        # the two chunk-0-column product launches of a column-split step as ONE paired launch (False: two launches)
        self.pair_phase0 = True
        del col
        if not keep_plain:
            del m
        if self.exchange == "allgather":
            self.send = torch.zeros(C, self.L, dtype=torch.float32, device=dev)  # tails of short chunks stay 0
        self.bufs = [torch.zeros(self.n_pad, dtype=torch.float32, device=dev) for _ in range(2)]

    CHUNK0_FRAC = 0.4

    def chunk_rows(self, c: int) -> tuple[int, int]:
        """Local rows [a, b) of row chunk c on this rank."""
        return min(self.cb[c], self.rows), min(self.cb[c + 1], self.rows)

    def _chunk_of(self, lr: torch.Tensor) -> torch.Tensor:
        """Row chunk of local rows lr (any rank's: the boundaries are the same on every rank)."""
        inner = torch.tensor(self.cb[1:-1], dtype=lr.dtype, device=lr.device)
        return torch.searchsorted(inner, lr, right=True)

    # ---- ghost layout (set-up: one exchange of the index lists)
    def _ghost_layout(self, col: torch.Tensor) -> torch.Tensor:
        """Builds the compact chunk-major / owner-minor layout, the per-(chunk, peer) send and receive lists, and
        returns `col` renumbered into the layout."""
        ctx, W, r, C, L, dev = self.ctx, self.ctx.world, self.ctx.rank, self.chunks, self.L, self.ctx.device
        cuts_t = torch.tensor(self.cuts, dtype=torch.int64, device=dev)
        need = torch.unique(col.long())  # ascending global ids = owner-major
        owner = torch.searchsorted(cuts_t[1:], need, right=True)
        need, owner = need[owner != r], owner[owner != r]  # ghosts (own rows are all kept)
        chunk = self._chunk_of(need - cuts_t[owner])
        # receive side: ghost (chunk c, owner q) counts; own segment of chunk c = own rows of chunk c
        cnt = torch.bincount(chunk * W + owner, minlength=C * W).view(C, W).cpu()
        own = [b - a for a, b in (self.chunk_rows(c) for c in range(C))]
        for c in range(C):
            cnt[c, r] = own[c]
        # chunk c = [ghosts of every peer q != r, in rank order | own rows of chunk c]: the ghost part is ONE
        # contiguous all_to_all_single output whose per-peer regions follow rank order (self region empty)
        self.recv_counts = cnt.tolist()  # [c][q]
        self.seg, self.ghost0, self.ghost_len, off = [0] * (C * W), [0] * C, [0] * C, 0
        for c in range(C):
            self.ghost0[c] = off
            for q in [q for q in range(W) if q != r] + [r]:
                self.seg[c * W + q] = off  # segment (c, q) starts here
                off += self.recv_counts[c][q]
            self.ghost_len[c] = self.seg[c * W + r] - self.ghost0[c]
        self.n_pad = max(1, off)
        # layout position of every ghost: its segment start + rank among the ghosts of that segment (ascending g)
        key = chunk * W + owner
        order = torch.sort(key * (self.n + 1) + need).indices  # stable (c, q, g) order
        pos = torch.empty_like(need)
        seg_dev = torch.tensor(self.seg, dtype=torch.int64, device=dev)
        ks = key[order]
        first = torch.searchsorted(ks, ks, right=False)  # index of the first ghost of the same segment
        pos[order] = seg_dev[ks] + (torch.arange(ks.numel(), device=dev) - first)
        # renumber the local columns: own rows -> own segment of their chunk, ghosts -> pos
        g = col.long()
        mine = (g >= self.row0) & (g < self.row1)
        lo = (g - self.row0).clamp(0, max(0, self.rows - 1))  # (only own columns use own_pos)
        lch = self._chunk_of(lo)
        cb_dev = torch.tensor(self.cb, dtype=torch.int64, device=dev)
        own_pos = seg_dev[lch * W + r] + (lo - cb_dev[lch])
        gpos = pos[torch.searchsorted(need, g).clamp(max=max(0, need.numel() - 1))] if need.numel() else g
        out = torch.where(mine, own_pos, gpos).to(torch.int32)
        self.ghost_ids, self.ghost_pos = need, pos
        self.send_idx, self.send_counts, self.sendbuf = [torch.zeros(0, dtype=torch.int32, device=dev)] * C, \
            [[0] * W for _ in range(C)], [torch.zeros(0, device=dev)] * C
        self.send_csr = None
        if ctx.distributed:  # (a Context without a process group only emulates one rank's products)
            # send side: tell every owner which of its rows this rank needs (counts, then ids, owner-major)
            dev_c = dev if ctx.backend == "nccl" else torch.device("cpu")
            req_counts = torch.bincount(owner, minlength=W).to(dev_c)
            got_counts = torch.empty_like(req_counts)
            dist.all_to_all_single(got_counts, req_counts)
            got = torch.empty(int(got_counts.sum()), dtype=torch.int64, device=dev_c)
            dist.all_to_all_single(got, need.to(dev_c), got_counts.tolist(), req_counts.tolist())
            got = got.to(dev) - self.row0  # local rows peer q needs, ascending per peer
            peer = torch.repeat_interleave(torch.arange(W, device=dev), got_counts.to(dev))
            gchunk = self._chunk_of(got)
            self.send_idx, self.send_counts = [], []
            for c in range(C):
                sel = gchunk == c  # owner-major order kept: peers in rank order, rows ascending
                # layout positions, int32: the pack kernel reads 4 B of index per entry (ops.gather_)
                self.send_idx.append((got[sel] - self.cb[c] + self.seg[c * W + r]).to(torch.int32).contiguous())
                self.send_counts.append(torch.bincount(peer[sel], minlength=W).tolist())
            self.sendbuf = [torch.empty(ix.numel(), dtype=torch.float32, device=dev) for ix in self.send_idx]
            # the same send lists inverted per own row (send_ptr: CSR over the chunk's rows, send_slot: slots in
            # sendbuf[c]): the sliced product's fused combine writes each row's value into its slots itself
            self.send_csr = []
            for c in range(C):
                a_c, b_c = self.chunk_rows(c)
                rows_c = b_c - a_c
                lr = (self.send_idx[c].long() - self.seg[c * W + r])
                order = torch.sort(lr, stable=True).indices
                ptr = torch.zeros(rows_c + 1, dtype=torch.int64, device=dev)
                if rows_c:
                    ptr[1:] = torch.bincount(lr, minlength=rows_c).cumsum(0)
                self.send_csr.append((ptr.to(torch.int32).contiguous(), order.to(torch.int32).contiguous()))
        self.n_ghost = int(need.numel())
        return out

    @staticmethod
    def powerlaw(ctx: Context, n_rows: int, nnz: int, alpha: float = 2.5, seed: int = 1,
                 slices: int = 0, head: float = 0.0625, balance: float = 0.0,
                 chunks: int | None = None, item_nnz: int = 0, exchange: str = "ghost",
                 keep_plain: bool = False, colsplit: bool | None = None,
                 chunk0_frac: float | None = None) -> DistributedSpMV:
        rp = powerlaw_row_ptr(n_rows, nnz, alpha, seed)
        cuts = nnz_balanced_cuts(rp, ctx.world)
        local = powerlaw_csr_rows(rp, cuts[ctx.rank], cuts[ctx.rank + 1], n_rows, seed)
        return DistributedSpMV(ctx, rp, local, cuts, slices, head, balance, chunks, item_nnz, exchange, keep_plain,
                               colsplit, chunk0_frac)

    def vendor_matrix(self) -> torch.Tensor:
        """This rank's rows as a torch sparse CSR tensor (layout columns): `torch.mv(A, xp)` runs hipSPARSE."""
        if self.plain is None:
            raise ValueError("built without keep_plain=True")
        m = self.plain
        return torch.sparse_csr_tensor(m.row_ptr.to(torch.int32), m.col, m.val, size=(m.n_rows, m.n_cols))

    @property
    def local_nnz(self) -> int:
        return sum(p.nnz for _, _, p in self.parts)

    # ---- layout conversion (natural global order <-> local layout)
    def layout_ids(self) -> torch.Tensor:
        """Global id of every local-layout entry (-1: padding), int64 [n_pad]."""
        dev = self.ctx.device
        if self.exchange == "allgather":
            ids = torch.full((self.n_pad,), -1, dtype=torch.int64, device=dev)
            ids[self.colmap] = torch.arange(self.n, device=dev)
            return ids
        ids = torch.full((self.n_pad,), -1, dtype=torch.int64, device=dev)
        ids[self.local_positions()] = torch.arange(self.row0, self.row1, device=dev)
        ids[self.ghost_pos] = self.ghost_ids
        return ids

    def to_padded(self, x: torch.Tensor) -> torch.Tensor:
        """x (natural order, full) -> this rank's layout vector."""
        x = x.to(self.ctx.device, torch.float32)
        if self.exchange == "allgather":
            xp = torch.zeros(self.n_pad, dtype=torch.float32, device=self.ctx.device)
            xp[self.colmap] = x
            return xp
        xp = torch.zeros(self.n_pad, dtype=torch.float32, device=self.ctx.device)
        xp[self.local_positions()] = x[self.row0:self.row1]
        xp[self.ghost_pos] = x[self.ghost_ids]  # the entries the exchange delivers, taken from the full x here
        return xp

    def from_padded(self, xp: torch.Tensor) -> torch.Tensor:
        """Layout vector -> full natural-order vector (ghost layout: own rows all-gathered; tests / inspection)."""
        if self.exchange == "allgather":
            return xp[self.colmap]
        mine = xp[self.local_positions()]
        if not self.ctx.distributed:
            return mine.clone()
        return self._gather_rows(mine)

    def _gather_rows(self, own: torch.Tensor) -> torch.Tensor:
        """This rank's rows (local order) of a vector -> the full natural-order vector (one all-gather; collective)."""
        if not self.ctx.distributed:
            return own
        buf = torch.zeros(self.block, dtype=own.dtype, device=own.device)
        buf[:own.numel()] = own
        parts = self.ctx.all_gather(buf)
        return torch.cat([p[:self.cuts[q + 1] - self.cuts[q]] for q, p in enumerate(parts)])

    def local_positions_chunk(self, c: int) -> torch.Tensor:
        a, b = self.chunk_rows(c)
        s0 = self.seg[c * self.ctx.world + self.ctx.rank]
        return torch.arange(s0, s0 + (b - a), device=self.ctx.device)

    def local_positions(self) -> torch.Tensor:
        """Layout positions of this rank's rows, in local row order."""
        if self.exchange == "allgather":
            return self.colmap[self.row0:self.row1]
        return torch.cat([self.local_positions_chunk(c) for c in range(self.chunks)])

    # ---- products
    def _mul(self, part, xp: torch.Tensor, dst: torch.Tensor) -> None:
        if self.sliced:
            part.spmv(xp, dst)
        elif isinstance(part, ColSplitCSR):
            dst.copy_(part.product(xp))
        else:
            dst.copy_(spmv(part, xp))

    def _send(self, c: int, part) -> tuple | None:
        """The fused pack of chunk c (send_ptr, send_slot, sendbuf) when its product is a sliced one, else None."""
        if not self.sliced or self.send_csr is None or self.exchange != "ghost" or not self.fuse_pack:
            return None
        ptr, slot = self.send_csr[c]
        return (ptr, slot, self.sendbuf[c])

    def _post_chunk(self, out: torch.Tensor, c: int, packed: bool = False):
        """Ghost exchange of chunk c: pack this rank's send entries (one index_select), then ONE collective
        (Context.exchange: a list all_to_all on RCCL, the per-peer sends/receives grouped over the xGMI links) whose
        per-peer receive entries are views of the chunk's ghost region (segments in rank order), so the entries
        land in place. One collective call instead of a batch of per-peer P2P ops keeps the N = 8 step off the
        host-launch bound (scripts/host_overhead_lab.py)."""
        W, r = self.ctx.world, self.ctx.rank
        if self.send_idx[c].numel() and not packed:
            gather_(out, self.send_idx[c], self.sendbuf[c])
        if not self.comm:
            return []
        if self._segs[c] is None:  # per-peer segments of the send buffer and of the chunk's ghost region (fixed)
            soff, scnt, roff, rcnt, so = [], [], [], [], 0
            for q in range(W):
                ns = 0 if q == r else self.send_counts[c][q]
                soff.append(so), scnt.append(ns)
                so += ns
                roff.append(self.seg[c * W + q]), rcnt.append(0 if q == r else self.recv_counts[c][q])
            self._segs[c] = (soff, scnt, roff, rcnt)
        soff, scnt, roff, rcnt = self._segs[c]
        return self.ctx.exchange_segments(c, self.sendbuf[c], soff, scnt, out, roff, rcnt)

    def _wait(self, k: int) -> None:
        for w in self._pending[k]:
            w.wait()
        self._pending[k] = []

    def finish(self) -> None:
        """Waits for the exchanges a column-split step left in flight (the next step waits for them itself; call this
        before reading the layout vector a step returned)."""
        self._wait(0)
        self._wait(1)

    def _step_colsplit(self, xp: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """Column-split schedule (2 chunks): products over the chunk-0 columns of xp (their exchange was posted
        mid-way through the previous step) for both row chunks, then — once the previous step's chunk-1 exchange has
        landed — the chunk-1 columns, the combine of row chunk c and the post of its exchange. Nothing waits at the
        end of the step: the chunk-1 exchange overlaps the next step's chunk-0-column products, so in steady state
        no exchange is exposed (4 product launches per step instead of 2)."""
        W, r = self.ctx.world, self.ctx.rank
        self._wait(0)
        (a0, b0, p0), (a1, b1, p1) = self.parts
        if self.pair_phase0 and b0 > a0 and b1 > a1 and isinstance(p0, SlicedCSR) and isinstance(p1, SlicedCSR) \
                and p0.cr is not None and p1.cr is not None and p0.n_slices + p1.n_slices <= 64:
            # both row chunks' chunk-0-column products in ONE launch (a launch of a few items per wave pays its ramp
            # and tail once: scripts/spmv_host_lab.py, profiles/r5_spmv/)
            h0, h1 = p0.n_slices // 16, p1.n_slices // 16
            p0.products_pair(p1, xp, (0, h0), (0, h1), mode=p0.phase_blocks[0] << 8)
        else:
            for c, (a, b, part) in enumerate(self.parts):
                if b > a:
                    part.product_phase(xp, 0, c)
        self._wait(1)
        pending = [[], []]
        for c, (a, b, part) in enumerate(self.parts):
            s0 = self.seg[c * W + r]
            send = self._send(c, part) if b > a else None
            if b > a:
                if send is not None:
                    part.product_phase(xp, 1, c, out[s0:s0 + (b - a)], send=send)
                else:
                    part.product_phase(xp, 1, c, out[s0:s0 + (b - a)])
            pending[c] = self._post_chunk(out, c, packed=send is not None)
        self._pending = pending
        return out

    def step_padded(self, xp: torch.Tensor, defer_exchange: bool = False) -> torch.Tensor:
        """xp (this rank's layout) -> A xp in the same layout (own rows + every ghost the next product reads).
        The result lives in one of two internal buffers; the buffer that is not `xp` is overwritten.
        defer_exchange (column split): return with the last chunk's exchange still in flight — the next step waits
        for it before the products that read those columns (an iterating caller: the steady-state pipeline); call
        finish() before reading the result yourself."""
        out = self.bufs[0] if xp.data_ptr() != self.bufs[0].data_ptr() else self.bufs[1]
        if self.colsplit and self.ctx.distributed:
            self._step_colsplit(xp, out)
            if not defer_exchange:
                self.finish()
            return out
        W, L, works = self.ctx.world, self.L, []
        for c, (a, b, part) in enumerate(self.parts):
            if self.exchange == "allgather":
                dst = out[c * L:c * L + (b - a)] if not self.ctx.distributed else self.send[c, :b - a]
            else:
                s0 = self.seg[c * W + self.ctx.rank]
                dst = out[s0:s0 + (b - a)]
            send = self._send(c, part) if b > a and self.ctx.distributed else None
            if b > a:
                if send is not None:
                    part.spmv(xp, dst, send=send)  # product + combine + fix-up + pack
                else:
                    self._mul(part, xp, dst)
            if not self.ctx.distributed:
                continue
            if self.exchange == "allgather":
                if self.comm:
                    works.append(dist.all_gather_into_tensor(out[c * W * L:(c + 1) * W * L], self.send[c],
                                                             async_op=True))
            else:
                works += self._post_chunk(out, c, packed=send is not None)
        for w in works:
            w.wait()
        return out

    def bytes_sent_per_step(self) -> float:
        """Payload bytes this rank sends per step: its ghost entries for every peer (ghost), or its padded chunk to
        every peer (allgather)."""
        W, r = self.ctx.world, self.ctx.rank
        if not self.ctx.distributed:
            return 0.0
        if self.exchange == "allgather":
            return 4.0 * self.chunks * self.L * (W - 1)
        return 4.0 * sum(cnt[q] for cnt in self.send_counts for q in range(W) if q != r)

    def step(self, x: torch.Tensor) -> torch.Tensor:
        """x (full, natural order, replicated) -> A x (full, natural order, replicated)."""
        y = self.step_padded(self.to_padded(x))
        self.finish()
        return self.from_padded(y)

    def iterate(self, xp: torch.Tensor, steps: int, defer: bool = True) -> torch.Tensor:
        """x <- A x, `steps` times, in this rank's layout (the power-iteration pattern the schedule is built for): each
        step's output is the next step's input, and with `defer` (column split) each step's chunk-1 exchange is still
        in flight when the next step starts its chunk-0-column products. Returns the last layout vector (one of the two
        internal buffers) with every exchange finished."""
        for _ in range(steps):
            xp = self.step_padded(xp, defer_exchange=defer)
        self.finish()
        return xp

    def iterate_reference(self, xp: torch.Tensor, steps: int) -> torch.Tensor:
        """fp64 A^steps xp in this rank's layout (own rows and every ghost), the oracle of iterate(): each step
        multiplies this rank's rows in fp64 and all-gathers the WHOLE vector (no ghost exchange, no column split, no
        deferral involved). Collective."""
        ids = self.layout_ids()
        m = ids >= 0
        cur = xp.double()
        for _ in range(steps):
            full = self._gather_rows(self.reference_local(cur))
            cur = torch.zeros(self.n_pad, dtype=torch.float64, device=xp.device)
            cur[m] = full[ids[m]]
        return cur

    def iterate_max_rel_err(self, xp: torch.Tensor, steps: int, defer: bool = True, reduce: bool = True) -> float:
        """Max error of EVERY layout entry after `steps` iterated steps (iterate) against iterate_reference, relative
        to the largest reference entry. Both runs (and their collectives) come first; reduce=False: this rank's value
        only."""
        got = self.iterate(xp, steps, defer).double()
        want = self.iterate_reference(xp, steps)
        m = self.layout_ids() >= 0
        scale = want[m].abs().max().clamp_min(1e-300) if bool(m.any()) else torch.ones((), dtype=torch.float64)
        err = ((got[m] - want[m]).abs().max() / scale).item() if bool(m.any()) else 0.0
        return self.ctx.max_over_ranks(err) if reduce else err

    def reference_local(self, xp: torch.Tensor) -> torch.Tensor:
        """fp64 product of this rank's rows with xp (its layout), in local row order."""
        outs = []
        for a, b, part in self.parts:
            if isinstance(part, ColSplitCSR):
                outs.append(part.reference(xp))
            elif isinstance(part, SlicedCSR):
                outs.append(part.reference(xp))
            else:
                rows = torch.repeat_interleave(torch.arange(part.n_rows, device=xp.device),
                                               (part.row_ptr[1:] - part.row_ptr[:-1]).to(xp.device))
                y = torch.zeros(part.n_rows, dtype=torch.float64, device=xp.device)
                y.index_add_(0, rows, part.val.double().to(xp.device) * xp.double()[part.col.long().to(xp.device)])
                outs.append(y)
        return torch.cat(outs) if outs else torch.zeros(0, dtype=torch.float64, device=xp.device)

    def layout_max_rel_err(self, y: torch.Tensor, xp: torch.Tensor, reduce: bool = True) -> float:
        """Max relative error of EVERY entry of the layout vector y = A xp against fp64: own rows and the ghost
        entries the exchange delivered (each compared with its owner's fp64 row, gathered once), i.e. the
        product and the exchange that the timed step performs. Same value on every rank (reduce=False: this
        rank's entries only, no collective after the all-gather of the fp64 rows)."""
        self.finish()
        full = self._gather_rows(self.reference_local(xp))
        ids = self.layout_ids()
        m = ids >= 0
        got, want = y[m].double(), full[ids[m]]
        scale = full.abs().max().clamp_min(1e-30) if full.numel() else torch.ones((), dtype=torch.float64)
        err = ((got - want).abs().max() / scale).item() if want.numel() else 0.0
        return self.ctx.max_over_ranks(err) if reduce else err

