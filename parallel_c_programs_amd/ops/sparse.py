"""Sparse matrix-vector products.

Reference parity: create_csr_matrix / multiply_naive / multiply (banded, implicit columns) / compare of
3-serial-optimization/spmv.c. GPU: CSR-adaptive nnz-balanced kernel (any degree distribution, incl. the
north-star 1e8-nnz power-law graph) and a banded kernel without column indices.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from .._native import cpu_lib, ops


@dataclass
class CSR:
    row_ptr: torch.Tensor  # int64 [n_rows + 1]
    col: torch.Tensor      # int32 [nnz]
    val: torch.Tensor      # float32 [nnz]
    n_cols: int
    items: torch.Tensor | None = None  # GPU work items (int64 [k, 3]), built by plan()

    @property
    def n_rows(self) -> int:
        return self.row_ptr.numel() - 1

    @property
    def nnz(self) -> int:
        return self.val.numel()

    def to(self, device) -> "CSR":
        return CSR(self.row_ptr.to(device), self.col.to(device), self.val.to(device), self.n_cols,
                   None if self.items is None else self.items.to(device))

    def plan(self) -> "CSR":
        """CSR-adaptive analysis (host, once per matrix): rows -> nnz-balanced work items."""
        from .. import _C  # noqa: F401  (pybind module carries the planner)

        items = _C.spmv_csr_plan(self.row_ptr.cpu().contiguous())
        self.items = items.to(self.row_ptr.device)
        return self

    def row_block(self, r0: int, r1: int) -> "CSR":
        """Rows [r0, r1) as their own CSR (views of col/val; the work-item plan is rebuilt on demand)."""
        a, b = int(self.row_ptr[r0]), int(self.row_ptr[r1])
        return CSR((self.row_ptr[r0:r1 + 1] - a).contiguous(), self.col[a:b], self.val[a:b], self.n_cols)

    def dense(self) -> torch.Tensor:
        rows = torch.repeat_interleave(torch.arange(self.n_rows, device=self.val.device),
                                       (self.row_ptr[1:] - self.row_ptr[:-1]).to(self.val.device))
        d = torch.zeros(self.n_rows, self.n_cols, dtype=torch.float32, device=self.val.device)
        d.index_put_((rows, self.col.long()), self.val, accumulate=True)
        return d


class PackedLayoutUnavailable(ValueError):
    """SlicedCSR: the requested item size needs the packed index stream, which this matrix's slices cannot use."""


class SlicedCSR:
    """XCD-sliced CSR for SpMV on MI355X (csrc/kernels/spmv.hip: spmv_sliced_kernel).

    The columns are cut into ``n_slices`` (8 x phases) ranges of about equal nnz; slice s keeps its nonzeros
    contiguous (slice-major copy of col/val, row order kept) and its own nnz-balanced work items over the rows it
    TOUCHES (rows with >= 1 nonzero in the slice); ``lrow`` holds, per nonzero, the offset of its row among the
    item's touched rows. The kernel deals slice s to the workgroups that share one XCD, so each 4-MiB L2 only
    holds one slice's part of x, and writes one compact partial per touched row (``ypart``, slice-major); the
    combine pass sums each row's partials using ``row_mask`` (bit s: slice s touches the row) and ``chunk_base``
    (touched rows of each slice before every 64-row chunk). ``head``: the lowest-index columns holding that
    fraction of the nonzeros (the hottest of a power-law graph) are dealt to the slices by row blocks instead,
    so every XCD keeps its own copy of them. Same product as the plain CSR kernel (fp32 sums in a different,
    fixed order). Built once per matrix on the matrix's device (torch ops; the item cuts use the host planner).
    """

    def __init__(self, m: CSR, n_slices: int = 16, head: float = 0.0625, balance: float = 0.0, item_nnz: int = 1024,
                 pack: bool = True, col_split: int = 0):
        from .. import _C  # noqa: F401  (pybind module carries the planner)

        if n_slices % 8 or not 8 <= n_slices <= 32:
            raise ValueError("n_slices must be 8, 16, 24 or 32")
        if item_nnz not in (256, 384, 512, 1024):
            raise ValueError("item_nnz must be 256, 384, 512 or 1024 (4, 6, 8 or 16 nonzeros per lane)")
        self.item_nnz = item_nnz
        # kernel layout bits: items of 512 nonzeros (bit 1), of 256 (bit 27) or 384 (bit 28; both packed layout only)
        self.mode = {512: 2, 256: 1 << 27, 384: 1 << 28}.get(item_nnz, 0)
        dev = m.val.device
        n, S, nnz = m.n_rows, n_slices, m.nnz
        self.n_rows, self.n_cols, self.n_slices, self.nnz = n, m.n_cols, S, nnz
        col = m.col.to(dev)
        hist = torch.bincount(col, minlength=m.n_cols).double()
        H = int(torch.searchsorted(hist.cumsum(0), torch.tensor([head * nnz], device=dev, dtype=torch.float64))) \
            if head > 0 else 0
        if col_split:  # column split: slices 0 .. S/2-1 cover columns [0, col_split), the others [col_split, n_cols)
            if S % 16 or not 0 < col_split < m.n_cols:
                raise ValueError("col_split needs 16 or 32 slices and 0 < col_split < n_cols")
            H = min(H, col_split)
        self.head_cols, self.col_split = H, int(col_split)
        # slice bounds over the tail: equal quantiles of a per-column cost = nnz in the column + balance * mean
        # nnz per column (balance 0: equal nnz per slice, the measured best)
        w = hist + balance * nnz / max(1, m.n_cols)
        w[:H] = 0
        cum = w.cumsum(0)
        if col_split:
            S2, B = S // 2, int(col_split)
            t0, tot = float(cum[B - 1]), float(cum[-1])
            g = torch.arange(1, S2, device=dev, dtype=torch.float64)
            b0 = torch.searchsorted(cum, g * (t0 / S2), right=True).clamp(max=B)
            b1 = torch.searchsorted(cum, t0 + g * ((tot - t0) / S2), right=True).clamp(min=B)
            bounds = torch.cat([b0, torch.tensor([B], device=dev), b1]).to(torch.int32)
        else:
            tgt = torch.arange(1, S, device=dev, dtype=torch.float64) * (float(cum[-1]) / S)
            bounds = torch.searchsorted(cum, tgt, right=True).to(torch.int32)
        self.bounds = bounds.cpu()
        if item_nnz in (256, 384):  # decided BEFORE the build: these items exist in the packed index stream only
            b = self.bounds.tolist()
            widest = max(h - l for l, h in zip([0] + b, b + [m.n_cols]))
            if not pack or nnz == 0 or H >= 1 << 21 or widest >= 1 << 21:
                raise PackedLayoutUnavailable(f"item_nnz {item_nnz} needs the packed index stream (every slice < 2^21 "
                                              f"columns; widest {widest})")
        sid = torch.bucketize(col, bounds, right=True)  # slice of every nonzero (int64)
        deg = (m.row_ptr[1:] - m.row_ptr[:-1]).to(dev)
        rows = torch.repeat_interleave(torch.arange(n, device=dev), deg)
        if H > 0:  # head nonzeros: by row blocks of equal head nnz
            inh = col < H
            hrows = rows[inh]
            hcum = torch.bincount(hrows, minlength=n).cumsum(0).double()
            rcut = torch.searchsorted(hcum, torch.arange(1, S, device=dev, dtype=torch.float64) * (float(hcum[-1]) / S),
                                      right=True)
            sid[inh] = torch.bucketize(hrows, rcut, right=True)
            del inh, hrows, hcum
        order = torch.sort(sid, stable=True).indices
        self.col = col[order].contiguous()
        self.val = m.val.to(dev)[order].contiguous()
        counts = torch.bincount(sid * n + rows, minlength=S * n).view(S, n)
        del order, rows, sid, col
        slice_nnz = counts.sum(1).cpu()
        if int(slice_nnz.max()) >= 2 ** 31:
            raise ValueError("a slice holds >= 2^31 nonzeros: use more slices")
        nz0 = torch.zeros(S, dtype=torch.int64)
        nz0[1:] = slice_nnz.cumsum(0)[:-1]
        n_chunks = (n + 63) // 64
        mask = torch.zeros(n, dtype=torch.int64, device=dev)
        base = torch.zeros(n_chunks, S, dtype=torch.int32, device=dev)
        items, fix, item0, out0 = [], [], [0], [0]
        self.lrow = torch.empty(nnz, dtype=torch.int16, device=dev)
        for k in range(S):
            touched = counts[k] > 0
            trows = torch.nonzero(touched).flatten()  # the rows slice k touches, ascending
            tcnt = counts[k][trows]
            mask |= touched.long() << k
            csum = touched.int().cumsum(0, dtype=torch.int32)
            base[1:, k] = csum[63:64 * (n_chunks - 1):64]  # touched rows before row 64c
            rp = torch.zeros(trows.numel() + 1, dtype=torch.int64, device=dev)
            rp[1:] = tcnt.cumsum(0)
            rpc = rp.cpu()
            it = _C.spmv_csr_plan(rpc, item_nnz)  # items over the compact (touched) rows (rows <= nnz per item)
            r0, r1 = it[:, 0] & 0xFFFFFFFF, it[:, 0] >> 32
            # a later piece of a split long row: a single-row item not starting at the row's first nonzero;
            # encoded as an empty row range (row1 == row0), its sum goes to extra[] and is fixed up into y
            idx = torch.nonzero(((r1 - r0) == 1) & (it[:, 1] != rpc[r0])).flatten()
            fix.append(torch.stack([idx + item0[-1], trows.cpu()[r0[idx]]], 1))
            it[idx, 0] = r0[idx] | (r0[idx] << 32)
            items.append(it)
            item0.append(item0[-1] + it.shape[0])
            out0.append(out0[-1] + trows.numel())
            nzk = int(rpc[-1])
            if nzk:  # offset of every nonzero's row among its item's touched rows (< kItemRows = 1023)
                itd = it.to(dev)
                row_of = torch.repeat_interleave(torch.arange(trows.numel(), device=dev), tcnt)
                item_of = torch.repeat_interleave(torch.arange(itd.shape[0], device=dev), itd[:, 2] - itd[:, 1])
                off = (row_of - (itd[:, 0] & 0xFFFFFFFF)[item_of]).clamp_(min=0)
                self.lrow[int(nz0[k]):int(nz0[k]) + nzk] = off.to(torch.int16)
                del itd, row_of, item_of, off
            del touched, trows, tcnt, csum, rp
        del counts
        self.items = torch.cat(items).to(dev)
        fix = torch.cat(fix)
        fix = fix[torch.sort(fix[:, 1], stable=True).indices]  # by row, item order kept: deterministic fix-up sums
        self.fix = fix.to(torch.int32).contiguous().to(dev)
        # fix range of every 64-row combine chunk (the fused combine's fix-up epilogue): entries [fc[c], fc[c + 1])
        n_ch = (n + 63) // 64
        self.fix_chunk0 = torch.searchsorted(self.fix[:, 1].contiguous().long(),
                                             torch.arange(0, n_ch + 2, device=dev) * 64).to(torch.int32).contiguous()
        # combine + fix-up (+ pack) in ONE launch (True) or the in-library two-launch form (False, the default: faster
        # for a single matrix, 69 + 5 us against 77 us on the 1e8-nnz product; DistributedSpMV turns it on for its
        # distributed steps, where the send-buffer pack rides along: profiles/r5_spmv/)
        self.fused_combine = False
        # resident product blocks per CU of the column-split phase 0 / phase 1 launches (0: the library default, 3;
        # DistributedSpMV sets them by rank size)
        self.phase_blocks = (0, 0)
        self.row_mask = mask.to(torch.int32).contiguous()  # bit 31 wraps into the sign: read as u32 on device
        self.chunk_base = base.contiguous()
        self.meta = torch.cat([nz0, torch.tensor(item0, dtype=torch.int64), torch.tensor(out0, dtype=torch.int64)])
        self.meta = self.meta.contiguous()
        self.ypart = torch.empty(max(1, out0[-1]), dtype=torch.float32, device=dev)
        self.extra = torch.empty(max(1, item0[-1]), dtype=torch.float32, device=dev)
        self._pack(slice_nnz, pack)
        assert item_nnz not in (256, 384) or self.cr is not None  # (decided above)

    def _pack(self, slice_nnz: torch.Tensor, pack: bool) -> None:
        """Packed index stream (the kernel's production layout): one int32 per nonzero = column - first tail column
        of its slice (bits 0-20; a head column is stored as itself with bit 21 set) | row offset in the item << 22.
        4 B instead of 4 + 2 B of index traffic per nonzero and one load instruction fewer per element. Used when
        every slice spans < 2^21 columns (1e7 columns / 16 slices: widest 1.8M); otherwise the unpacked arrays."""
        S, H = self.n_slices, self.head_cols
        b = self.bounds.tolist()
        lo, hi = [0] + b, b + [self.n_cols]
        self.colbase = lo
        self.cr = None
        if not pack or self.nnz == 0 or H >= 1 << 21 or max(h - l for l, h in zip(lo, hi)) >= 1 << 21:
            return
        dev = self.col.device
        sid = torch.repeat_interleave(torch.arange(S, device=dev), slice_nnz.to(dev))
        c = self.col.long()
        w = torch.where(c < H, c | (1 << 21), c - torch.tensor(lo, device=dev)[sid]) | (self.lrow.long() << 22)
        self.cr = (w - ((w >> 31) << 32)).to(torch.int32)  # two's-complement wrap of the 32-bit word

    @property
    def partials(self) -> int:
        """Compact partials per product (touched (row, slice) pairs)."""
        return int(self.meta[-1])

    def products_pair(self, other: SlicedCSR, x: torch.Tensor, phases: tuple[int, int],
                      other_phases: tuple[int, int], mode: int = 0) -> None:
        """The products (no combine) of phases `phases` = (lo, n) of this matrix and `other_phases` of `other` (another
        sliced matrix over the same x) in ONE launch; each matrix then combines its own partials as after a
        products-only call (the distributed column-split step's two row chunks, chunk-0 columns)."""
        for m in (self, other):
            if m.cr is None:
                raise ValueError("products_pair: packed index stream only")
            if getattr(m, "_meta_packed", None) is None:
                m._meta_packed = torch.cat([m.meta, torch.tensor(m.colbase, dtype=torch.int64)]).contiguous()
                m._no_lrow = torch.empty(0, dtype=torch.int16, device=m.cr.device)
        if self.mode != other.mode:
            raise ValueError("products_pair: both matrices need the same item size")
        item_mode = 4 if self.mode & (1 << 27) else 6 if self.mode & (1 << 28) else self.mode
        ops().spmv_sliced_pair(x, item_mode, int(mode), self.cr, self.val, self.items, self._meta_packed, self.ypart,
                               self.extra, self.n_slices, int(phases[0]), int(phases[1]), other.cr, other.val,
                               other.items, other._meta_packed, other.ypart, other.extra, other.n_slices,
                               int(other_phases[0]), int(other_phases[1]))

    def combine(self, out: torch.Tensor, send: tuple | None = None) -> torch.Tensor:
        """The combine + split-row fix-up of the partials the last products-only call wrote, into out[:n_rows], in ONE
        launch; send = (send_ptr, send_slot, sendbuf): also write every row's value into the send-buffer slots that
        carry it to the peers (the distributed step's pack, fused into the same launch)."""
        meta = self._meta_packed if getattr(self, "_meta_packed", None) is not None else self.meta
        sp, ss, sb = send if send is not None else (None, None, None)
        if send is not None:
            self._check_send(sp, ss, sb)
        ops().spmv_sliced_combine(self.ypart, self.row_mask, self.chunk_base, meta, self.n_slices, self.extra,
                                  self.fix, self.fix_chunk0, out, self.n_rows, sp, ss, sb)
        return out

    def _check_send(self, sp: torch.Tensor, ss: torch.Tensor, sb: torch.Tensor) -> None:
        """The fused pack writes sendbuf[send_slot[k]] for k in [send_ptr[r], send_ptr[r + 1]) of every row r, on the
        device, unchecked: the lists are validated here once per set (a host sync; the distributed step reuses the
        same tensors every step). send_ptr: n_rows + 1 non-decreasing entries from 0 to len(send_slot); every slot
        inside sendbuf."""
        key = (sp.data_ptr(), ss.data_ptr(), sb.data_ptr(), sp.numel(), ss.numel(), sb.numel())
        if key in getattr(self, "_send_ok", ()):
            return
        if sp.numel() < self.n_rows + 1 or sp.dtype != torch.int32 or ss.dtype != torch.int32:
            raise ValueError("send: int32 send_ptr of n_rows + 1 entries and int32 send_slot")
        p = sp[:self.n_rows + 1].long()
        ok = int(p[0]) == 0 and int(p[-1]) == ss.numel() and bool((p[1:] >= p[:-1]).all())
        if ss.numel():
            ok = ok and int(ss.min()) >= 0 and int(ss.max()) < sb.numel()
        if not ok:
            raise ValueError("send: send_ptr must rise from 0 to len(send_slot) and every slot must lie in sendbuf")
        self._send_ok = getattr(self, "_send_ok", set()) | {key}

    def spmv(self, x: torch.Tensor, out: torch.Tensor | None = None, mode: int = 0,
             phases: tuple[int, int] | None = None, send: tuple | None = None) -> torch.Tensor:
        """y = A x; `out` (contiguous f32, >= n_rows elements) receives y in place when given. mode bit 4: products
        only (compact partials, no combine), bit 5: combine + fix-up only (of the partials a bit-4 call wrote).
        phases=(lo, n): the products of slices [8 lo, 8 (lo + n)) only (one slice per XCD per phase) — with col_split,
        phases (0, S/16) multiply the columns below the split and (S/16, S/16) the others. A combining call runs the
        fused combine (combine + fix-up in one launch, and the send-buffer pack when `send` is given; see combine())."""
        if self.fused_combine and not (mode & 16) and (mode & ~32 & 0xCF) == 0 and self.cr is not None:
            if out is None:
                out = torch.empty(self.n_rows, dtype=torch.float32, device=x.device)
            if not (mode & 32):
                self.spmv(x, mode=mode | 16, phases=phases)
            return self.combine(out, send)
        if send is not None:
            raise ValueError("send: the fused combine only (production layout)")
        if phases is not None:
            lo, n = phases
            if not (0 <= lo and 0 < n and lo + n <= self.n_slices // 8):
                raise ValueError(f"phases {phases} outside the {self.n_slices // 8} phases")
            mode |= (lo << 16) | (n << 21)
        # production: packed index stream (bit 6: ballot combine, 8+: resident blocks, 16-25: phases, 26: nt partials)
        if self.cr is not None and (mode & 0x8F) == 0:
            if getattr(self, "_meta_packed", None) is None:
                self._meta_packed = torch.cat([self.meta, torch.tensor(self.colbase, dtype=torch.int64)]).contiguous()
                self._no_lrow = torch.empty(0, dtype=torch.int16, device=self.cr.device)
            return ops().spmv_sliced(self._no_lrow, self.cr, self.val, x, self.items, self.row_mask, self.chunk_base,
                                     self.fix, self._meta_packed, self.ypart, self.extra, self.n_rows, out,
                                     8 | self.mode | mode)
        return ops().spmv_sliced(self.lrow, self.col, self.val, x, self.items, self.row_mask, self.chunk_base, self.fix,
                                 self.meta, self.ypart, self.extra, self.n_rows, out, mode | self.mode)

    def touched_rows(self, k: int) -> torch.Tensor:
        """Rows slice k touches (ascending), from the row mask."""
        return torch.nonzero((self.row_mask.long() >> k) & 1).flatten()

    def rows(self) -> torch.Tensor:
        """Row of every stored nonzero, rebuilt from the items, lrow and the row mask (the layout the kernel reads)."""
        it = self.items
        r0 = it[:, 0] & 0xFFFFFFFF
        S = self.n_slices
        out = torch.empty(self.nnz, dtype=torch.int64, device=it.device)
        for k in range(S):
            a, b = int(self.meta[S + k]), int(self.meta[S + k + 1])
            base = int(self.meta[k])
            itk = it[a:b]
            item_of = torch.repeat_interleave(torch.arange(b - a, device=it.device), itk[:, 2] - itk[:, 1])
            nzk = int(item_of.numel())
            trows = self.touched_rows(k).to(it.device)
            out[base:base + nzk] = trows[r0[a:b][item_of] + self.lrow[base:base + nzk].long()]
        return out

    def reference(self, x: torch.Tensor) -> torch.Tensor:
        """fp64 product straight from the sliced layout (tests the layout on any device). Row sums are segment
        reductions over the row-sorted products (an fp64 index_add_ serialises on a power-law graph's hot rows:
        ~10 s at 1e8 nnz on the GPU)."""
        rows = self.rows().to(x.device)
        order = torch.sort(rows, stable=True).indices
        prod = (self.val.double().to(x.device) * x.double()[self.col.long().to(x.device)])[order]
        lengths = torch.bincount(rows, minlength=self.n_rows)
        return torch.segment_reduce(prod, "sum", lengths=lengths, unsafe=True)


class _CSRStruct(ctypes.Structure):
    _fields_ = [("n_row_ptr", ctypes.c_int), ("row_ptr", ctypes.POINTER(ctypes.c_int)),
                ("col_ind", ctypes.POINTER(ctypes.c_int)), ("n_values", ctypes.c_int),
                ("values", ctypes.POINTER(ctypes.c_float))]


def banded_csr(n: int, a: int, b: int, c: int, d: int, e: int, seed: int | None = 1) -> CSR:
    """The reference's 5-band matrix (create_csr_matrix, spmv.c:74-144) built by the host C library: same
    structure and, under glibc, the same rand() value stream (seed 1 = the reference's unseeded default;
    seed=None continues the current C rand() sequence)."""
    lib = cpu_lib()
    if seed is not None:
        lib.srand(int(seed))
    lib.create_csr_matrix.restype = ctypes.POINTER(_CSRStruct)
    lib.create_csr_matrix.argtypes = [ctypes.c_int] * 7
    lib.free_csr_matrix.argtypes = [ctypes.POINTER(_CSRStruct)]
    m = lib.create_csr_matrix(n, n, a, b, c, d, e)
    s = m.contents
    nnz = s.n_values
    rp = torch.tensor(_as_array(s.row_ptr, n + 1, ctypes.c_int), dtype=torch.int64)
    col = torch.from_numpy(_np_view(s.col_ind, nnz, "int32").copy())
    val = torch.from_numpy(_np_view(s.values, nnz, "float32").copy())
    lib.free_csr_matrix(m)
    return CSR(rp, col, val, n)


def _np_view(ptr, n, dtype):
    import numpy as np

    return np.ctypeslib.as_array(ptr, shape=(n,)).view(dtype) if n else np.zeros(0, dtype=dtype)


def _as_array(ptr, n, ctype):
    return _np_view(ptr, n, "int32").astype("int64")


def create_vector(n: int) -> torch.Tensor:
    """rand()/RAND_MAX vector of the reference (spmv.c:148-154)."""
    lib = cpu_lib()
    lib.create_vector.restype = ctypes.POINTER(ctypes.c_float)
    lib.create_vector.argtypes = [ctypes.c_int]
    p = lib.create_vector(n)
    v = torch.from_numpy(_np_view(p, n, "float32").copy())
    lib.pcmx_free(ctypes.cast(p, ctypes.c_void_p))
    return v


def powerlaw_csr(n_rows: int, target_nnz: int, alpha: float = 2.5, seed: int = 1, n_cols: int | None = None) -> CSR:
    """Synthetic power-law graph (Chung-Lu style): Zipf row degrees (exponent 1/(alpha-1)) on a permuted row
    order, sorted columns drawn from a Zipf column density. Generated by the multithreaded host C library."""
    n_cols = n_rows if n_cols is None else n_cols
    lib = cpu_lib()
    rp = torch.empty(n_rows + 1, dtype=torch.int64)
    nnz = lib.pcmx_powerlaw_row_counts(n_rows, int(target_nnz), float(alpha), int(seed), rp.data_ptr())
    col = torch.empty(nnz, dtype=torch.int32)
    val = torch.empty(nnz, dtype=torch.float32)
    lib.pcmx_powerlaw_fill(n_rows, n_cols, rp.data_ptr(), int(seed), col.data_ptr(), val.data_ptr())
    return CSR(rp, col, val, n_cols)


def powerlaw_row_ptr(n_rows: int, target_nnz: int, alpha: float = 2.5, seed: int = 1) -> torch.Tensor:
    """Row pointer of powerlaw_csr (cheap: O(n_rows)); every rank computes it to partition by nnz."""
    rp = torch.empty(n_rows + 1, dtype=torch.int64)
    cpu_lib().pcmx_powerlaw_row_counts(n_rows, int(target_nnz), float(alpha), int(seed), rp.data_ptr())
    return rp


def powerlaw_csr_rows(row_ptr: torch.Tensor, row0: int, row1: int, n_cols: int, seed: int = 1) -> CSR:
    """Rows [row0, row1) of powerlaw_csr (bit-identical), generated without materialising the rest."""
    base = int(row_ptr[row0])
    nnz = int(row_ptr[row1]) - base
    col = torch.empty(nnz, dtype=torch.int32)
    val = torch.empty(nnz, dtype=torch.float32)
    cpu_lib().pcmx_powerlaw_fill_rows(int(row0), int(row1), int(n_cols), row_ptr.data_ptr(), int(seed),
                                      col.data_ptr(), val.data_ptr())
    return CSR((row_ptr[row0:row1 + 1] - base).contiguous(), col, val, n_cols)


def spmv(m: CSR, x: torch.Tensor) -> torch.Tensor:
    """y = A x (float32)."""
    if x.is_cuda:
        if m.items is None or m.items.device != x.device:
            m.plan()
        return ops().spmv_csr(m.row_ptr, m.col, m.val, x, m.items)
    y = torch.empty(m.n_rows, dtype=torch.float32)
    rp32 = m.row_ptr.to(torch.int32).contiguous()
    cpu_lib().pcmx_spmv_csr_omp(m.n_rows, rp32.data_ptr(), m.col.data_ptr(), m.val.data_ptr(),
                                x.contiguous().data_ptr(), y.data_ptr())
    return y


def spmv_banded(vals: torch.Tensor, row_off: torch.Tensor, n: int, a: int, b: int, c: int, d: int, e: int,
                x: torch.Tensor, variant: int = 8) -> torch.Tensor:
    """Banded product with implicit columns (the reference's s_matrix `multiply`, spmv.c:212-329). GPU variant 8
    (default): each 16-row block's values as one aligned 16-B stream, x band windows in LDS (falls back to variant 1
    when the geometry or alignment rules it out); 1: row blocks with 4-B value loads and in-register band limits;
    0: one wave per row."""
    if x.is_cuda:
        return ops().spmv_banded(vals, row_off, int(n), int(a), int(b), int(c), int(d), int(e), x, int(variant))

    class SMat(ctypes.Structure):
        _fields_ = [("values", ctypes.c_void_p), ("n", ctypes.c_int), ("a", ctypes.c_int), ("b", ctypes.c_int),
                    ("c", ctypes.c_int), ("d", ctypes.c_int), ("e", ctypes.c_int)]

    sm = SMat(vals.data_ptr(), n, a, b, c, d, e)
    y = torch.empty(n, dtype=torch.float32)
    lib = cpu_lib()
    lib.multiply.argtypes = [ctypes.POINTER(SMat), ctypes.c_void_p, ctypes.c_void_p]
    lib.multiply(ctypes.byref(sm), x.contiguous().data_ptr(), y.data_ptr())
    return y
