"""Distributed 2-D 5-point stencil — north-star config "16384^2 bf16 + halo exchange" (ancestor: the
1-cell halo exchange of ref 2-mpi-region-growing/region.c:250-353).

Decomposition: row slabs (rows split near-evenly over the ranks, full width per rank). On xGMI a row slab
needs only TWO contiguous halo rows per step (one per neighbour link, 2 x cols x 2 B = 64 KiB at 16384
columns) instead of four strided edges for a 2-D grid — fewer, larger, contiguous messages, each on its
own point-to-point link.

Overlap: the halo exchange is posted as one grouped RCCL send/recv (RCCL runs it on its own stream);
the interior rows, which do not read the halo, are computed on the compute stream meanwhile; only the
boundary rows wait for the halo, and both boundary bands are updated by ONE launch (two row spans). Measured on
one rank's slab (scripts/stencil_rank_lab.py, profiles/r2_stencil/rank_lab.txt): one edge launch instead of two
saves 8-16 us per step at N=2-8; issuing it on a side stream to run beside the interior kernel was 5% faster at
N=8 but up to 17% slower at N=2/4 (cross-stream waits), so it stays on the compute stream.

Temporal blocking (fuse=T in 2, 3, 4, 6, 8): the slab keeps T halo rows per side, one grouped exchange moves
T rows per neighbour every T updates (1/T of the messages — the halos are latency-bound on xGMI), and one
fused kernel performs the T updates with a single HBM read + write per cell. Bit-identical to fuse=1.
Deep halo (halo_mult m): mT halo rows exchanged every m steps, the rows next to a neighbour computed redundantly in
between (StencilSlab docstring): one exchange and one edge launch per m steps.
"""
from __future__ import annotations

import torch

from ..ops.stencil import DEFAULT_K, FUSED_STEPS, init_grid, stencil5_fused_spans_, stencil5_fused_step_, stencil5_step_
from .dist import Context
from .topology import split


def auto_fuse(slab_rows: int) -> int:
    """Fused updates per kernel for a rank's slab height: the fused kernel is VALU-bound and every wave recomputes
    its T-row trapezoid overlap, so deep fusion pays on tall slabs and short slabs want shallower fusion. Measured as
    the distributed step shape (interior launch + the two-span edge launch, 16384 columns, round-3 lane geometries:
    4 columns per lane at T >= 6 below 12288 rows, 2-row edge waves; scripts/stencil_lanes_lab.py,
    profiles/r3_stencil/lanes_*.txt), GLUP/s: 16384 rows T=8 5.5k; 8192 T=8 4.9k / T=6 4.8k; 4096 T=6 4.4k / T=8 4.2k
    / T=4 3.9k; 2048 T=6 3.4k / T=8 3.3k / T=4 3.3k. Re-checked in round 6 with the current kernel and deep halo
    (profiles/r6_stencil/t6_t8_ab.txt): 2048 rows T=6 deep5 3.65-3.76k / T=8 3.41-3.72k; 4096 T=6 4.39-4.45k /
    T=8 4.32-4.38k."""
    return 8 if slab_rows >= 6144 else 6


def auto_halo_mult(slab_rows: int, fuse: int, world: int) -> int:
    """Halo depth in units of `fuse` rows (the deep-halo schedule, see StencilSlab): 5 on distributed slabs of up to
    4096 rows, 1 otherwise. Measured per step of one interior rank (scripts/stencil_rank_lab.py, T = 6): round 4
    (profiles/r4_stencil/rank_lab_deep_halo.txt, rank_lab_deep3.txt): 2048 rows (N = 8) interior + edge launch every
    step 0.0595-0.0603 ms, m = 2 0.0550-0.0624, m = 3 0.0581; 8192 rows 0.163 -> 0.175 with m = 2 (taller slabs lose:
    their two-launch step hides the edge launch better than the extended launches cost). Round 5, m swept 3..8 in one
    process (profiles/r5_stencil/halo_depth_sweep.txt and the A/B files beside it): 2048 rows m = 3 0.0569-0.0581,
    m = 4 0.0552-0.0559, m = 5 0.0549, m = 6 0.0569, m = 8 0.0563; with 18 rows per wave (rpw_deep_ab.txt, 6
    alternations) m = 4 0.0547, m = 5 0.0539; 4096 rows (N = 4) edge launch every step 0.0966, m = 3 0.0955, m = 4
    0.0902, m = 5 0.0893, m = 8 0.0893 (another box, rpw_n4_ab.txt: m = 4 0.0957, m = 5 0.0928). A timed window of a
    multiple of 5 steps (the bench's 10 / 20) holds whole periods whatever step it starts at. At 8192 rows (N = 2, T = 8)
    depth does not matter (halo_depth_n2_n8_n1.txt)."""
    return 5 if world > 1 and fuse > 1 and 10 * fuse <= slab_rows <= 4096 else 1


class StencilSlab:
    """One rank's (rows + 2 halo, cols) bf16 slab and its double buffer.

    Deep halo (halo_mult m >= 2, fuse T > 1): the slab keeps H = mT halo rows per side and exchanges H rows every
    m steps (every mT updates). The exchange step computes T updates over its own rows AND the (m-1)T halo rows
    next to each neighbour (their T-step cone reaches H rows out: exactly the received halo); the next step then
    already holds T valid halo rows and updates rows -(m-2)T .. rows + (m-2)T with ONE launch and no exchange, and so
    on down to 0 extra rows at the m-th step. Per m steps: one exchange of mT rows, one interior launch + one edge
    launch (the two halo-dependent bands, mT rows each) and m-1 full launches — instead of m exchanges and 2m
    launches; the redundant rows cost (m-1)mT / rows of extra work (0.6% at m = 2, T = 6, 2048 rows). Bit-identical
    to single steps: every computed row follows the same arithmetic from the same inputs."""

    def __init__(self, ctx: Context, n: int, cols: int | None = None, k: float = DEFAULT_K, fuse: int = 1,
                 halo_mult: int = 1, pattern: str = "random"):
        self.ctx, self.n, self.cols, self.k = ctx, n, (n if cols is None else cols), k
        if fuse != 1 and fuse not in FUSED_STEPS:
            raise ValueError(f"fuse: 1 or one of {FUSED_STEPS} updates per kernel")
        if halo_mult < 1 or (halo_mult > 1 and fuse == 1):
            raise ValueError("halo_mult: >= 1, and > 1 only with fused steps")
        self.fuse = fuse
        self.m = halo_mult if ctx.distributed else 1
        self.halo = fuse * self.m  # T fused updates read T rows beyond the slab; m steps read mT
        self.row0, row1 = split(n, ctx.world, ctx.rank)
        self.rows = row1 - self.row0
        if self.rows < 2 * self.halo:
            raise ValueError(f"each rank needs at least {2 * self.halo} rows")
        self.pattern = pattern
        self.u = init_grid(self.rows, self.cols, self.row0, n, device=ctx.device, halo=self.halo, pattern=pattern)
        # explicit launch shapes (ops.stencil.launch_shape; 0 = the production rule) of the full / interior launches
        # and of the two-span edge launch: lab sweeps set them per slab, nothing process-global
        self.shape, self.edge_shape = 0, 0
        self.v = self.u.clone()
        self.steps_done = 0
        self.phase = 0  # step index within the current deep-halo period (0: the exchange step)
        self.north = ctx.rank - 1 if ctx.rank > 0 else -1
        self.south = ctx.rank + 1 if ctx.rank < ctx.world - 1 else -1

    def _post_exchange(self):
        """One grouped exchange of `halo` contiguous boundary rows per neighbour (Context.neighbour_exchange: ONE
        list all_to_all on RCCL, ~19 us of host time against ~60 us for a batch of four P2P ops, which would make a
        2048-row slab's step, ~45 us of GPU time at N = 8, launch-bound)."""
        u, h, rows, W, cols = self.u, self.halo, self.rows, self.ctx.world, self.cols
        # as segments of the flat slab (Context.exchange_segments: the native RCCL path on a GPU job, else the same
        # views through one list all-to-all); slot 4 (the SpMV chunks use 0 and 1)
        soff, scnt, roff, rcnt = [0] * W, [0] * W, [0] * W, [0] * W
        if self.north >= 0:
            soff[self.north], scnt[self.north], roff[self.north], rcnt[self.north] = h * cols, h * cols, 0, h * cols
        if self.south >= 0:
            q = self.south
            soff[q], scnt[q], roff[q], rcnt[q] = rows * cols, h * cols, (rows + h) * cols, h * cols
        flat = u.view(-1)
        return self.ctx.exchange_segments(4, flat, soff, scnt, flat, roff, rcnt)

    def _extent(self, phase: int) -> tuple[int, int]:
        """Local rows the step at `phase` updates: its own rows plus (m-1-phase)T halo rows on each side with a
        neighbour."""
        e = (self.m - 1 - phase) * self.fuse
        return (-e if self.north >= 0 else 0), self.rows + (e if self.south >= 0 else 0)

    def _update(self, u, v, row_range=None):
        """`fuse` updates u -> v over local rows row_range (default all)."""
        if self.fuse > 1:
            stencil5_fused_step_(u, v, self.row0, self.n, self.k, halo=self.halo, steps=self.fuse, row_range=row_range,
                                 shape=self.shape)
        else:
            stencil5_step_(u, v, self.row0, self.n, self.k, row_range=row_range)

    def _update_edges(self, u, v, lo: int, hi: int):
        """The two halo-dependent bands [lo, T) and [rows - T, hi) after the halo rows arrived: one launch."""
        T, rows = self.fuse, self.rows
        if self.fuse > 1:
            stencil5_fused_spans_(u, v, ((lo, T), (rows - T, hi)), self.row0, self.n, self.k, halo=self.halo,
                                  steps=self.fuse, shape=self.edge_shape)
        else:
            stencil5_step_(u, v, self.row0, self.n, self.k, row_range=(0, T))
            stencil5_step_(u, v, self.row0, self.n, self.k, row_range=(rows - T, rows))

    def step(self, overlap: bool = True, comm: bool = True) -> None:
        """Advances `fuse` time steps: at phase 0 one halo exchange overlapped with the interior launch, then the
        edge launch; at later phases of a deep halo, one launch and no exchange. comm=False (bench attribution only):
        the same launches with the exchange skipped (the halo rows go stale: the grid is no longer checkable)."""
        ctx, rows, T = self.ctx, self.rows, self.fuse  # rows within T of a rank edge read the halo
        if not ctx.distributed:
            self._update(self.u, self.v)
        elif self.phase == 0:
            lo, hi = self._extent(0)
            if overlap and rows > 2 * T:
                reqs = self._post_exchange() if comm else []
                self._update(self.u, self.v, (T, rows - T))
                for r in reqs:
                    r.wait()
                self._update_edges(self.u, self.v, lo, hi)
            else:
                for r in (self._post_exchange() if comm else []):
                    r.wait()
                self._update(self.u, self.v, (lo, hi))
        else:
            self._update(self.u, self.v, self._extent(self.phase))
        self.u, self.v = self.v, self.u
        self.steps_done += T
        self.phase = (self.phase + 1) % self.m

    def halo_bytes_per_step(self) -> float:
        """Bytes this rank sends per step: `halo` rows of `cols` bf16 to each neighbour every m steps."""
        if not self.ctx.distributed:
            return 0.0
        nbrs = (self.north >= 0) + (self.south >= 0)
        return nbrs * self.halo * self.cols * self.u.element_size() / self.m

    # ---- checkpoint / resume: each rank writes its own slab; tensors only (weights_only load)
    def checkpoint(self, prefix: str) -> str:
        path = f"{prefix}.rank{self.ctx.rank}-of-{self.ctx.world}.pt"
        torch.save({"u": self.interior().cpu(), "row0": self.row0, "rows": self.rows, "n": self.n, "cols": self.cols,
                    "k": self.k, "steps_done": self.steps_done}, path)
        self.ctx.barrier()
        return path

    def restore(self, prefix: str) -> None:
        path = f"{prefix}.rank{self.ctx.rank}-of-{self.ctx.world}.pt"
        st = torch.load(path, map_location="cpu", weights_only=True)
        if (st["row0"], st["rows"], st["n"], st["cols"]) != (self.row0, self.rows, self.n, self.cols):
            raise ValueError(f"checkpoint {path} does not match this decomposition")
        self.interior().copy_(st["u"].to(self.u.device))  # halos are refreshed by the next exchange
        self.v.copy_(self.u)
        self.k, self.steps_done = st["k"], st["steps_done"]
        self.phase = 0  # the next step exchanges (the restored halo rows are stale)

    def run(self, steps: int, overlap: bool = True, graph: bool = False) -> torch.Tensor:
        """`steps` updates (a multiple of `fuse`). graph=True (single GPU rank): a HIP graph of two launches
        (u->v->u, 2*fuse updates) is captured once and replayed, removing per-launch host overhead."""
        f = self.fuse
        if steps % f:
            raise ValueError(f"steps must be a multiple of fuse={f}")
        if graph and self.ctx.device.type == "cuda" and not self.ctx.distributed and steps >= 2 * f:
            fresh = getattr(self, "_g", None) is None or self._g_ptr != (self.u.data_ptr(), self.v.data_ptr())
            g = self._graph()
            if fresh:  # building the graph ran one eager pair of launches
                steps -= 2 * f
            for _ in range(steps // (2 * f)):
                g.replay()
            self.steps_done += 2 * f * (steps // (2 * f))
            steps %= 2 * f
        for _ in range(steps // f):
            self.step(overlap)
        return self.u

    def _graph(self):
        if getattr(self, "_g", None) is None or self._g_ptr != (self.u.data_ptr(), self.v.data_ptr()):
            stream = torch.cuda.Stream()
            stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(stream):  # warm-up outside capture (lazy init of the op)
                self._update(self.u, self.v)
                self._update(self.v, self.u)
            torch.cuda.current_stream().wait_stream(stream)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._update(self.u, self.v)
                self._update(self.v, self.u)
            self._g, self._g_ptr = g, (self.u.data_ptr(), self.v.data_ptr())
            self.steps_done += 2 * self.fuse  # the warm-up pair advanced the state
        return self._g

    def interior(self) -> torch.Tensor:
        return self.u[self.halo:self.halo + self.rows]

    def gather(self) -> torch.Tensor | None:
        """Full (n, cols) grid on root."""
        if not self.ctx.distributed:
            return self.interior().clone()
        mine = self.interior().contiguous()
        if self.ctx.is_root:
            parts = [mine]
            for r in range(1, self.ctx.world):
                a, b = split(self.n, self.ctx.world, r)
                buf = torch.empty((b - a, self.cols), dtype=mine.dtype, device=mine.device)
                self.ctx.recv(buf, r)  # (host-staged on the gloo test transport: Context.recv)
                parts.append(buf)
            return torch.cat(parts)
        self.ctx.send(mine, 0)
        return None


def reference_run(n: int, steps: int, cols: int | None = None, k: float = DEFAULT_K, device="cpu",
                  pattern: str = "random") -> torch.Tensor:
    """Single-domain run (the oracle the distributed result must equal bit for bit)."""
    cols = n if cols is None else cols
    u = init_grid(n, cols, 0, n, device=device, pattern=pattern)
    v = u.clone()
    for _ in range(steps):
        stencil5_step_(u, v, 0, n, k)
        u, v = v, u
    return u[1:-1]


def reference_run_torch(n: int, steps: int, cols: int | None = None, k: float = DEFAULT_K, device="cpu",
                        pattern: str = "random") -> torch.Tensor:
    """Single-domain run on plain PyTorch f32 ops (ops.stencil5_reference: no HIP kernel involved), the oracle of
    the bench's timed-grid check."""
    from ..ops.stencil import stencil5_reference

    cols = n if cols is None else cols
    u = init_grid(n, cols, 0, n, device=device, pattern=pattern)
    for _ in range(steps):
        u = stencil5_reference(u, 0, n, k)
    return u[1:-1]
