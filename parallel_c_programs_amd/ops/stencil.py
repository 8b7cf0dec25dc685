"""2-D 5-point stencil (explicit heat step) on bf16 slabs — north-star config "16384^2 bf16 + halo exchange".

    u'[i][j] = c + k * (((n + s) + (w + e)) - 4c),  f32 arithmetic (no contraction), bf16 (RNE) storage;
    the global boundary rows/columns are Dirichlet (copied).

A slab is a (rows + 2, cols) bf16 tensor: row 0 and row rows+1 are halo rows (neighbour ranks' boundary
rows, or unused at the global edge). Ancestor in the reference: the 4-neighbour update with a 1-cell halo of
2-mpi-region-growing/region.c:250-353, 499-527.
"""
from __future__ import annotations

import torch

from .._native import ops

DEFAULT_K = 0.2


def stencil5_reference(slab: torch.Tensor, global_row0: int, global_rows: int, k: float = DEFAULT_K) -> torch.Tensor:
    """Plain PyTorch f32 reference of one step on a slab (same operation order, bf16 rounding)."""
    u = slab.float()
    c = u[1:-1]
    n, s = u[:-2], u[2:]
    w = torch.roll(c, 1, dims=1)
    e = torch.roll(c, -1, dims=1)
    lap = ((n + s) + (w + e)) - 4.0 * c
    res = c + torch.tensor(k, dtype=torch.float32) * lap
    rows = torch.arange(slab.shape[0] - 2, device=slab.device) + global_row0
    fixed = (rows == 0) | (rows == global_rows - 1)
    res[fixed] = c[fixed]
    res[:, 0] = c[:, 0]
    res[:, -1] = c[:, -1]
    out = slab.clone()
    out[1:-1] = res.to(torch.bfloat16)
    return out


def stencil5_step_(u: torch.Tensor, out: torch.Tensor, global_row0: int = 0, global_rows: int | None = None,
                   k: float = DEFAULT_K, row_range: tuple[int, int] | None = None) -> torch.Tensor:
    """One step u -> out over local rows [r0, r1) (default: all). Halo rows of `out` are untouched."""
    rows = u.shape[0] - 2
    global_rows = rows if global_rows is None else global_rows
    r0, r1 = row_range or (0, rows)
    if u.is_cuda:
        ops().stencil5_(u, out, int(r0), int(r1), int(global_row0), int(global_rows), float(k))
        return out
    ref = stencil5_reference(u, global_row0, global_rows, k)
    out[1 + r0:1 + r1] = ref[1 + r0:1 + r1]
    return out


FUSED_STEPS = (2, 3, 4, 5, 6, 8)


def stencil5_fused_step_(u: torch.Tensor, out: torch.Tensor, global_row0: int = 0, global_rows: int | None = None,
                         k: float = DEFAULT_K, halo: int = 1, steps: int = 2,
                         row_range: tuple[int, int] | None = None, shape: int = 0) -> torch.Tensor:
    """`steps` fused updates u -> out (temporal blocking: one HBM read + write per cell per `steps` updates),
    bit-identical to `steps` stencil5_step_ calls. Slabs are (rows + 2*halo, cols); rows within `steps` of a
    rank boundary need halo >= steps (the halo rows must hold the neighbour's boundary rows). shape: an explicit
    launch shape for this launch (0: the production rule; see pcmx_stencil5xT_bf16_spans_shape; labs)."""
    rows = u.shape[0] - 2 * halo
    global_rows = rows if global_rows is None else global_rows
    r0, r1 = row_range or (0, rows)
    if u.is_cuda:
        ops().stencil5xT_(u, out, int(halo), int(steps), int(r0), int(r1), int(global_row0), int(global_rows), float(k),
                          int(shape))
        return out
    # CPU oracle: plain steps. A slab with h halo rows yields the next level on h-1 halo rows (its outermost
    # rows go stale); once h == 1 only global edges are allowed and the (unused) halo rows keep their values.
    cur, h = u, halo
    for _ in range(steps):
        nxt = stencil5_reference(cur, global_row0 - (h - 1), global_rows, k)
        if h > 1:
            cur, h = nxt[1:-1], h - 1
        else:
            cur = nxt
    out[halo + r0:halo + r1] = cur[h + r0:h + r1]
    return out


def stencil5_fused_spans_(u: torch.Tensor, out: torch.Tensor, spans, global_row0: int = 0,
                          global_rows: int | None = None, k: float = DEFAULT_K, halo: int = 1,
                          steps: int = 2, shape: int = 0) -> torch.Tensor:
    """`steps` fused updates over two disjoint local row spans [(a0, a1), (b0, b1)] in ONE kernel launch (the
    distributed step's two rank-edge bands once the halo has arrived); same results as one call per span."""
    (a0, a1), (b0, b1) = spans
    if u.is_cuda:
        rows = u.shape[0] - 2 * halo
        global_rows = rows if global_rows is None else global_rows
        ops().stencil5xT_spans_(u, out, int(halo), int(steps), int(a0), int(a1), int(b0), int(b1), int(global_row0),
                                int(global_rows), float(k), int(shape))
        return out
    for r in ((a0, a1), (b0, b1)):
        if r[1] > r[0]:
            stencil5_fused_step_(u, out, global_row0, global_rows, k, halo, steps, r)
    return out


def launch_shape(cpl: int = 0, rpw: int = 0, ahead: int = 0, paired: bool | None = None) -> int:
    """The `shape` word of an explicit stencil launch shape (each field 0 / None: the production rule's value).
    paired: True = paired waves (two vertically adjacent waves share their common trapezoid through LDS, round 6),
    False = independent waves."""
    if cpl not in (0, 4, 8) or not 0 <= rpw <= 255 or ahead not in (0, 3, 6, 9):
        raise ValueError("launch_shape: cpl 0/4/8, rpw 0..255, ahead 0/3/6/9")
    pair = 0 if paired is None else (1 if paired else 2)
    return cpl | (rpw << 8) | (ahead << 16) | (pair << 24)


def stencil5x2_step_(u, out, global_row0=0, global_rows=None, k=DEFAULT_K, halo=1, row_range=None):
    """Two fused updates (see stencil5_fused_step_)."""
    return stencil5_fused_step_(u, out, global_row0, global_rows, k, halo, 2, row_range)


def _hash32(x: torch.Tensor) -> torch.Tensor:
    """A 32-bit integer mix of int64 values in [0, 2^32) (two multiply-xorshift rounds). Every product stays below
    2^59, so the int64 arithmetic is exact and identical on the CPU and the GPU."""
    m = 0xFFFFFFFF
    x = ((x >> 16) ^ x) * 0x45D9F3B & m
    x = ((x >> 16) ^ x) * 0x45D9F3B & m
    return (x >> 16) ^ x


def init_grid(rows: int, cols: int, global_row0: int = 0, global_rows: int | None = None, device="cpu",
              halo: int = 1, pattern: str = "random", seed: int = 0) -> torch.Tensor:
    """Deterministic initial condition of the global grid, rows [global_row0 - halo, global_row0 + rows + halo).
    pattern "random" (default; the north star's random-init arrays): every cell uniform in [-1, 1) from a hash of its
    GLOBAL index (so any row-slab decomposition generates the same grid), the Dirichlet edge rows and columns
    included; pattern "hot": a hot top boundary row (1.0) and a hot square in the middle, 0 elsewhere. Rows outside
    the grid are 0."""
    global_rows = rows if global_rows is None else global_rows
    gi = torch.arange(global_row0 - halo, global_row0 + rows + halo, device=device).view(-1, 1)
    ci = torch.arange(cols, device=device).view(1, -1)
    if pattern == "random":
        idx = (gi.clamp_min(0) * cols + ci + (seed & 0xFFFF) * 0x9E3779B1) & 0xFFFFFFFF
        u = (_hash32(idx) & 0xFFFFFF).float() * (2.0 / (1 << 24)) - 1.0
    elif pattern == "hot":
        g, c = gi.float(), ci.float()
        hot = ((g - global_rows / 2).abs() < global_rows / 8) & ((c - cols / 2).abs() < cols / 8)
        u = torch.where(g == 0, torch.ones_like(hot, dtype=torch.float32), hot.float() * 0.5)
    else:
        raise ValueError("pattern: 'random' or 'hot'")
    u = torch.where((gi < 0) | (gi >= global_rows), torch.zeros_like(u), u)
    return u.to(torch.bfloat16).contiguous()
