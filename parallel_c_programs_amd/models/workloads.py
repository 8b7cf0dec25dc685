"""Step-able workloads with work models. Every workload owns its per-rank data (weak scaling unless noted),
exposes step() (one timed unit of work, including its collectives) and report(seconds, steps) (whole-job
throughput = sum over ranks), and check() (a numerics check against an independent reference)."""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import torch

from .. import ops
from ..parallel.collectives import global_scan
from ..parallel.dist import Context

# Pass threshold of every fp64-referenced numerics check (relative error): bench.py fails the run above it, and
# run_workload exits 1. Bit-exact checks (stencil, region growing, histogram) pass only when exact.
REL_ERR_LIMIT = 1e-5


@dataclass
class Workload:
    ctx: Context
    cfg: dict = field(default_factory=dict)
    name: str = ""
    unit: str = ""

    def step(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def work_per_step(self) -> float:
        """Units of work per step per rank (flops, bytes, updates...)."""
        raise NotImplementedError

    def scale(self) -> float:
        return 1e12 if self.unit == "TFLOPS" else 1e9

    def report(self, seconds: float, steps: int) -> dict:
        total = self.ctx.world * self.work_per_step() * steps / seconds / self.scale()
        return {"value": total, "unit": self.unit, "ms_per_step": 1e3 * seconds / steps}

    def check(self, reduce: bool = True) -> dict:
        """Numerics check against an independent reference: a dict with "check_passed" (bool) and the measured
        error(s). reduce=False returns THIS rank's values without the final reduction over ranks (bench.py merges
        them in its own collective decision step); every collective a check needs runs before its local-only part,
        so a local failure cannot leave another rank waiting in a data collective."""
        return {"check_passed": True}

    def compute_only_step(self) -> None:
        """The same kernels on the same data as step(), with every inter-rank exchange skipped (N > 1 attribution:
        full step minus this = the exposed communication; ref 2-mpi-region-growing/region.c:497-532 separates the
        exchange from the compute the same way). Leaves the workload's state unchecked: run it after check()."""
        self.step()

    def bytes_exchanged_per_step(self) -> float:
        """Payload bytes this rank SENDS to other ranks per step (averaged over a deep-halo period)."""
        return 0.0


class Sgemm(Workload):
    """C = A @ B, fp32 exact (MFMA v_mfma_f32_32x32x2_f32), per-rank operands (data-parallel, weak)."""

    def __init__(self, ctx, n=8192, variant=-1, **_):
        super().__init__(ctx, {"n": n, "variant": variant}, "sgemm", "TFLOPS")
        dev = ctx.device
        self.a = torch.empty(n, n, device=dev)
        self.b = torch.empty(n, n, device=dev)
        self.c = torch.empty(n, n, device=dev)
        ops.rand_uniform_(self.a, 1000 + ctx.rank)
        ops.rand_uniform_(self.b, 2000 + ctx.rank)
        self.n, self.variant = n, variant

    def step(self):
        if self.ctx.device.type == "cuda":
            ops.sgemm_out(self.a, self.b, self.c, variant=self.variant)
        else:
            torch.matmul(self.a, self.b, out=self.c)

    def work_per_step(self):
        return 2.0 * self.n ** 3

    def check(self, reduce: bool = True, block_rows: int = 2048):
        """EVERY element of the timed C against an fp64 GEMM of the same operands (row blocks of block_rows, so the
        fp64 copy of A is never whole), relative to max |C_ref| (ref 3-serial-optimization/spmv.c:179-191 compares
        every output too). Local only."""
        bd = self.b.double()
        err = torch.zeros((), dtype=torch.float64, device=self.a.device)
        big = torch.zeros((), dtype=torch.float64, device=self.a.device)
        for s in range(0, self.n, block_rows):
            ref = self.a[s:s + block_rows].double() @ bd
            err = torch.maximum(err, (self.c[s:s + block_rows].double() - ref).abs().max())
            big = torch.maximum(big, ref.abs().max())
            del ref
        del bd
        e = (err / big.clamp_min(1e-300)).item()
        if reduce:
            e = self.ctx.max_over_ranks(e)
        return {"max_rel_err_vs_fp64": e, "elements_checked": self.n * self.n, "check_passed": e <= REL_ERR_LIMIT}


class Reduce(Workload):
    """Global sum of world x n f32: local HBM-bound reduction + one-scalar RCCL all-reduce.

    With several ranks a step's all-reduce is left in flight on RCCL's stream and overlaps the NEXT step's local
    reduction: step k launches its reduction, then makes the compute stream wait for step k-1's all-reduce and stores
    that global total, then posts its own all-reduce. Every all-reduce is enqueued inside the step that computed its
    input and completes on the device before the bench's closing synchronize; settle() (called by check()) stores the
    last one's total."""

    def __init__(self, ctx, n=10**9, **_):
        super().__init__(ctx, {"n": n}, "reduce", "GB/s")
        self.x = torch.empty(int(n), device=ctx.device)
        ops.rand_uniform_(self.x, 3000 + ctx.rank, 0.0, 1.0)
        self.total = torch.zeros((), device=ctx.device)
        self._pending = None  # (work, partial sum) of the all-reduce still in flight
        self.overlap = os.environ.get("PCMX_REDUCE_OVERLAP", "1") != "0"  # 0: the round-5 blocking all-reduce

    def step(self):
        s = ops.reduce(self.x, "sum").reshape(1).float()
        if not self.ctx.distributed or not self.overlap:
            self.ctx.all_reduce_(s)
            self.total.copy_(s.reshape(()))
            return
        self.settle()
        self._pending = (self.ctx.all_reduce_async(s), s)

    def settle(self):
        """The compute stream waits for the all-reduce in flight (if any) and stores its global total."""
        if self._pending is not None:
            work, s = self._pending
            self._pending = None
            work.wait()
            self.total.copy_(s.reshape(()))

    def compute_only_step(self):
        self.settle()
        self.total.copy_(ops.reduce(self.x, "sum").reshape(()).float())

    def bytes_exchanged_per_step(self):
        return 4.0 if self.ctx.distributed else 0.0  # one f32 into the all-reduce

    def work_per_step(self):
        return 4.0 * self.x.numel()

    def check(self, reduce: bool = True):
        self.settle()
        ref = self.x.double().sum().reshape(1)
        self.ctx.all_reduce_(ref)  # (the one collective, before the local comparison)
        e = abs(self.total.item() - ref.item()) / max(abs(ref.item()), 1e-300)
        if reduce:
            e = self.ctx.max_over_ranks(e)
        return {"rel_err_vs_fp64": e, "check_passed": e <= REL_ERR_LIMIT}


class Axpy(Workload):
    """y <- alpha x + y over n f32 per GPU (the north star's AXPY hot loop; ref 6-opencl-region-growing/
    multiply_opencl.cl:1-4 is its element-wise ancestor): 12 B/element of HBM traffic per step, weak scaling, no
    communication. The ticket-ordered streaming kernel (csrc/kernels/vector.hip).

    The data make every step EXACT in fp32, so the timed output itself is checkable bit for bit after any number of
    steps: x = k / 2^11 (k < 2^11), y0 on the 2^-23 grid in [0, 1), alpha = 2^-12; every increment alpha x is then a
    multiple of 2^-23 and y stays below 2 (where that grid is representable) for fewer than 4096 steps."""

    ALPHA = 2.0 ** -12

    def __init__(self, ctx, n=10**9, **_):
        super().__init__(ctx, {"n": n, "alpha": self.ALPHA}, "axpy", "GB/s")
        self.x = torch.empty(int(n), device=ctx.device)
        self.y = torch.empty(int(n), device=ctx.device)
        ops.rand_uniform_(self.x, 5000 + ctx.rank, 0.0, 1.0)
        ops.rand_uniform_(self.y, 6000 + ctx.rank, 0.0, 1.0)
        self.x.mul_(2048.0).floor_().div_(2048.0)
        self.y.mul_(2.0 ** 23).floor_().div_(2.0 ** 23)
        self.y0 = self.y.clone()
        self.alpha, self.steps = self.ALPHA, 0

    def step(self):
        ops.axpy_(self.y, self.alpha, self.x)
        self.steps += 1

    def torch_step(self):
        """The same update through torch (the vendor bar); counted like a step."""
        self.y.add_(self.x, alpha=self.alpha)
        self.steps += 1

    def work_per_step(self):
        return 12.0 * self.x.numel()

    def check(self, reduce: bool = True, chunk: int = 1 << 26):
        """EVERY element of the timed output against fp64 y0 + steps * alpha * x (exact while steps < 4096), relative
        to max |y|. Local only."""
        err = torch.zeros((), dtype=torch.float64, device=self.x.device)
        big = torch.zeros((), dtype=torch.float64, device=self.x.device)
        n, a = self.x.numel(), self.steps * self.alpha
        for s0 in range(0, n, chunk):
            ref = self.y0[s0:s0 + chunk].double() + a * self.x[s0:s0 + chunk].double()
            err = torch.maximum(err, (self.y[s0:s0 + chunk].double() - ref).abs().max())
            big = torch.maximum(big, ref.abs().max())
        e = (err / big.clamp_min(1e-300)).item()
        if reduce:
            e = self.ctx.max_over_ranks(e)
        return {"rel_err_vs_fp64": e, "steps_applied": self.steps, "check_passed": e <= REL_ERR_LIMIT}


class Scan(Workload):
    """Inclusive prefix sum across ranks: local totals all-gathered, rank offset fed to the single-pass
    decoupled look-back scan as its initial value."""

    def __init__(self, ctx, n=10**9, **_):
        super().__init__(ctx, {"n": n}, "scan", "GB/s")
        self.x = torch.empty(int(n), device=ctx.device)
        ops.rand_uniform_(self.x, 4000 + ctx.rank, 0.0, 1.0)
        self.y = None

    def step(self):
        self.y = global_scan(self.x, self.ctx)

    def compute_only_step(self):
        self.y = global_scan(self.x, self.ctx, comm=False)

    def bytes_exchanged_per_step(self):
        return 4.0 if self.ctx.distributed else 0.0  # this rank's total into the all-gather

    def work_per_step(self):
        # effective bandwidth: the 8 B/element a scan must move (read + write); with several ranks the extra
        # 4 B/element reduce pass that seeds each rank's offset counts as time, not as work
        return 8.0 * self.x.numel()

    def check(self, reduce: bool = True, chunk: int = 1 << 26, one_rank_at_a_time: bool = False):
        """Every output of the timed scan (all n, not a prefix) against an fp64 cumsum carried across chunks, seeded
        with this rank's offset (the fp64 sum of the lower ranks' totals), and the look-back error word of the
        stream (lookback_ok False if any timed scan gave up a look-back). The totals' all-gather runs first: a rank
        whose stream reports a timed-out look-back still joins it, then reports the flag instead of raising.
        one_rank_at_a_time (ranks sharing one GPU): the ranks take turns for the fp64 cumsums, behind barriers.
        torch.cumsum is rocPRIM's look-back scan, which waits on blocks by index, and several processes' copies of it
        on one GPU can starve each other's predecessors."""
        tot = self.x.double().sum().reshape(1)
        totals = self.ctx.all_gather(tot)
        lookback_ok = True
        if self.x.is_cuda:
            try:
                ops.scan_check(self.x.device)
            except RuntimeError:
                lookback_ok = False
        carry = torch.zeros((), dtype=torch.float64, device=self.x.device)
        for t in totals[: self.ctx.rank]:
            carry = carry + t.to(carry.device).reshape(())
        err = torch.zeros((), dtype=torch.float64, device=self.x.device)
        n = self.x.numel()
        for turn in range(self.ctx.world if one_rank_at_a_time else 1):
            if one_rank_at_a_time and turn != self.ctx.rank:
                self.ctx.barrier()
                continue
            for s in range(0, n, chunk):
                ref = torch.cumsum(self.x[s:s + chunk].double(), 0) + carry
                err = torch.maximum(err, (self.y[s:s + chunk].double() - ref).abs().max())
                carry = ref[-1]
            if one_rank_at_a_time:
                if self.x.is_cuda:
                    torch.cuda.synchronize(self.x.device)
                self.ctx.barrier()
        # relative to this rank's largest prefix (its last one: the inputs are non-negative)
        e = (err / carry.abs().clamp_min(1e-30)).item()
        if reduce:
            e = self.ctx.max_over_ranks(e)
            lookback_ok = self.ctx.max_over_ranks(0.0 if lookback_ok else 1.0) == 0.0
        return {"rel_err_vs_fp64": e, "elements_checked": n, "lookback_ok": lookback_ok,
                "check_passed": e <= REL_ERR_LIMIT and lookback_ok}


class Stencil(Workload):
    """16384^2 bf16 5-point stencil, row slabs + halo exchange overlapped with the interior update.
    Strong scaling across ranks when `global_n` is fixed (the grid is split); weak when `per_rank`.
    fuse=T (default 0: auto_fuse of the slab height): T time steps per kernel (temporal blocking, bit-identical to single steps) and a T-row
    halo exchange every T steps; one step() then advances T time steps and counts T updates per cell."""

    def __init__(self, ctx, n=16384, per_rank=False, overlap=True, graph_steps=0, fuse=0, halo_mult=0,
                 pattern="random", **_):
        from ..parallel.stencil import StencilSlab, auto_fuse, auto_halo_mult

        rows = n * (ctx.world if per_rank else 1)
        fuse = int(fuse) or auto_fuse(rows // ctx.world)
        auto_m = not int(halo_mult)
        halo_mult = int(halo_mult) or auto_halo_mult(rows // ctx.world, fuse, ctx.world)
        self.ctx, self.overlap, self.pattern = ctx, overlap, pattern
        # The deep halo (m > 1) is proven on this job's own backend before it is timed: a small grid through the same
        # slab code at this world size must equal the single-domain oracle bit for bit; an AUTO depth that fails it
        # falls back to m = 1 (halo_selftest False in the line), an explicit one stays and fails the check.
        self.halo_selftest = None
        if halo_mult > 1 and ctx.distributed:
            self.halo_selftest = self._small_grid_ok(fuse, halo_mult)
            if not self.halo_selftest and auto_m:
                halo_mult = 1
        super().__init__(ctx, {"n": n, "rows": rows, "graph_steps": graph_steps, "fuse": fuse,
                               "halo_mult": halo_mult, "pattern": pattern}, "stencil", "GLUP/s")
        self.slab = StencilSlab(ctx, rows, n, fuse=fuse, halo_mult=halo_mult, pattern=pattern)
        self.graph_steps = graph_steps  # >0: one step() = graph_steps updates replayed from a HIP graph
        self.cells_local = self.slab.rows * n

    def step(self):
        if self.graph_steps:
            self.slab.run(self.graph_steps, self.overlap, graph=True)
        else:
            self.slab.step(self.overlap)

    def compute_only_step(self):
        self.slab.step(self.overlap, comm=False)

    def bytes_exchanged_per_step(self):
        return self.slab.halo_bytes_per_step()

    def work_per_step(self):
        return float(self.cells_local) * (self.graph_steps or self.slab.fuse)

    def report(self, seconds, steps):
        r = super().report(seconds, steps)
        # strong scaling (one fixed grid): the world-sum of local cells is the grid, not world x grid
        t = self.ctx.scalar(float(self.cells_local))
        self.ctx.all_reduce_(t)
        r["value"] = t.item() * (self.graph_steps or self.slab.fuse) * steps / seconds / 1e9
        return r

    def check(self, reduce: bool = True):
        """Two bit-exact checks.
        small grid: a small grid stepped through the same slab code at this world size (row slabs, fused T-row
          halo exchange, overlap) against the single-domain single-step oracle (collectives: it runs first);
        timed grid: the grid the timed steps produced (warm-up + timed, `steps_done` updates of the full 16384^2
          problem, this rank's rows) against a plain-PyTorch f32 single-step oracle of the whole grid
          (ops.stencil5_reference, bf16 rounding per step) run on this rank's device (local only)."""
        from ..parallel.stencil import reference_run_torch

        sl = self.slab
        ok = self._small_grid_ok(sl.fuse, sl.m)
        ref = reference_run_torch(sl.n, sl.steps_done, sl.cols, sl.k, device=self.ctx.device, pattern=self.pattern)
        mine = sl.interior()
        timed_ok = torch.equal(mine.view(torch.int16), ref[sl.row0:sl.row0 + sl.rows].view(torch.int16))
        del ref
        finite = bool(torch.isfinite(mine.float()).all())
        if reduce:
            timed_ok = self.ctx.max_over_ranks(0.0 if timed_ok else 1.0) == 0.0
            finite = self.ctx.max_over_ranks(0.0 if finite else 1.0) == 0.0
        return {"timed_grid_bit_exact": bool(timed_ok), "timed_grid_updates": sl.steps_done,
                "bit_exact_vs_single_step_oracle": bool(ok), "finite": bool(finite), "halo_selftest": self.halo_selftest,
                "check_passed": bool(timed_ok and ok and finite)}

    def _small_grid_ok(self, f: int, m: int) -> bool:
        """A small random grid stepped through the same slab code at this world size (row slabs, the fused / deep
        halo exchange, overlap) equals the single-domain single-step oracle bit for bit (collective; same answer on
        every rank)."""
        from ..parallel.stencil import StencilSlab, reference_run

        n, cols, steps = max(64, 2 * f * m * self.ctx.world + 8), 200, 4 * f * max(1, m)
        small = StencilSlab(self.ctx, n, cols, fuse=f, halo_mult=m, pattern=self.pattern)
        small.run(steps, self.overlap)
        full = small.gather()
        ok = 1.0
        if self.ctx.is_root:
            ref = reference_run(n, steps, cols, device=self.ctx.device, pattern=self.pattern)
            ok = float(torch.equal(full.view(torch.int16), ref.view(torch.int16)))
        return self.ctx.broadcast_(self.ctx.scalar(ok)).item() == 1.0


class SpMV(Workload):
    """Power-law CSR SpMV (nnz-balanced row blocks) + chunked exchange of y overlapped with the product
    (parallel/spmv.py): y <- A x in each rank's layout (own rows + ghosts by default, or the replicated padded
    layout with exchange="allgather"). Strong scaling: one fixed matrix."""

    def __init__(self, ctx, n_rows=10_000_000, nnz=100_000_000, alpha=2.5, slices=-1, head=0.0625,
                 balance=0.0, chunks=0, exchange="ghost", keep_plain=False, colsplit=None, **_):
        from ..parallel.spmv import DistributedSpMV

        slices = int(slices) if ctx.device.type == "cuda" else 0
        self.d = DistributedSpMV.powerlaw(ctx, n_rows, nnz, alpha, slices=slices, head=float(head),
                                          balance=float(balance), chunks=int(chunks) or None, exchange=exchange,
                                          keep_plain=keep_plain, colsplit=colsplit)
        slices = self.d.slices
        super().__init__(ctx, {"n_rows": n_rows, "nnz": nnz, "slices": slices, "head": head,
                               "chunks": self.d.chunks, "colsplit": self.d.colsplit}, "spmv", "GFLOP/s")
        x = ops.rand_uniform_(torch.empty(n_rows, device=ctx.device), 5, 0.0, 1.0)
        self.xp = self.d.to_padded(x)
        del x
        self.y = None
        # The column-split pipeline leaves each step's chunk-1 exchange in flight across the step boundary. Before it
        # is timed, the SAME job proves it on its own backend: ITERATE_STEPS chained steps x <- A x with the exchange
        # deferred must equal, bit for bit, the same steps with every exchange finished inside its step (same kernels,
        # same data: any difference is a missing wait). If they differ on any rank, the timed steps finish their
        # exchanges (defer off) and the line says so (pipeline_selftest False).
        self.defer, self.selftest = True, None
        if self.d.colsplit and ctx.distributed:
            a = self.d.iterate(self.xp, self.ITERATE_STEPS, defer=True).clone()
            b = self.d.iterate(self.xp, self.ITERATE_STEPS, defer=False)
            same = ctx.max_over_ranks(0.0 if torch.equal(a, b) else 1.0) == 0.0
            self.defer = self.selftest = same
            del a

    ITERATE_STEPS = 3

    def step(self):
        # the column-split pipeline: each step's last exchange overlaps the next step's first products (the next step
        # waits for it before the products that read those columns); check() finishes it
        self.y = self.d.step_padded(self.xp, defer_exchange=self.defer)

    def check(self, reduce: bool = True):
        """Every entry of the timed step's output layout (own rows AND the ghost entries the exchange wrote) against
        the fp64 product of its owner's row; then ITERATE_STEPS chained steps (each output the next input, exchanges
        deferred across step boundaries as in an iterating caller) against fp64 A^k x."""
        e = self.d.layout_max_rel_err(self.y, self.xp, reduce=reduce)
        self.y = None  # (iterate() reuses the output buffers)
        ei = self.d.iterate_max_rel_err(self.xp, self.ITERATE_STEPS, defer=self.defer, reduce=reduce)
        return {"max_rel_err_vs_fp64": e, "iterated_max_rel_err_vs_fp64": ei, "iterated_steps": self.ITERATE_STEPS,
                "pipeline_selftest": self.selftest, "deferred": self.defer and self.d.colsplit,
                "check_passed": e <= REL_ERR_LIMIT and ei <= REL_ERR_LIMIT}

    def compute_only_step(self):
        self.d.comm = False
        try:
            self.y = self.d.step_padded(self.xp, defer_exchange=self.defer)
        finally:
            self.d.comm = True

    def bytes_exchanged_per_step(self):
        return self.d.bytes_sent_per_step()

    def work_per_step(self):
        return 2.0 * self.d.local_nnz

    def report(self, seconds, steps):
        r = super().report(seconds, steps)
        nnz_all = self.d.local_nnz
        t = torch.tensor([float(nnz_all)], dtype=torch.float64, device=self.ctx.device)
        self.ctx.all_reduce_(t)
        r["value"] = 2.0 * t.item() * steps / seconds / 1e9  # strong scaling: fixed matrix, world-summed
        bytes_ = t.item() * 8 + self.d.n * 8 * 2
        r["effective_gbps"] = bytes_ * steps / seconds / 1e9
        return r


class Region3D(Workload):
    """3-D region growing on the reference volume (512^3, seed (50,300,300)), LDS-tiled kernel."""

    # T2: from the reference seed the region is exactly the box 0<x<100, 250<y<400, 250<z<400 of the
    # reference volume, whatever its noise background (ref 5-cuda-region-growing/raycast.cu:114-158, 281-318)
    BOX_VOXELS = 99 * 149 * 149  # 2,197,899

    def __init__(self, ctx, dim=512, method="tiled", **_):
        super().__init__(ctx, {"dim": dim}, "region3d", "Gvox/s")
        self.data = ops.create_volume(dim, device=ctx.device)
        self.method, self.region, self.launches = method, None, 0

    def step(self):
        self.region, self.launches = ops.region3d(self.data, method=self.method)

    def work_per_step(self):
        return float(self.data.numel())

    def check(self, reduce: bool = True):
        """The timed region: 2,197,899 voxels forming exactly the box (dim 512, the reference seed); other volume
        sizes against the serial CPU flood fill (csrc/cpu/oracles.c)."""
        got = self.region != 0
        voxels = int(got.sum())
        if self.data.shape[0] == 512:
            box = torch.zeros_like(got)
            box[251:400, 251:400, 1:100] = True  # [z][y][x]
            ok = voxels == self.BOX_VOXELS and torch.equal(got, box)
        else:
            ref, _ = ops.region3d(self.data.cpu())
            ok = torch.equal(got.cpu(), ref != 0)
        return {"region_voxels": voxels, "check_passed": bool(ok)}


class Raycast(Workload):
    def __init__(self, ctx, dim=512, image_dim=512, method="texture", **_):
        super().__init__(ctx, {"dim": dim, "image_dim": image_dim}, "raycast", "Grays/s")
        self.data = ops.create_volume(dim, device=ctx.device)
        self.region, _ = ops.region3d(self.data)
        self.image_dim, self.method = image_dim, method

    def step(self):
        self.image = ops.raycast(self.data, self.region, self.image_dim, method=self.method)

    def work_per_step(self):
        return float(self.image_dim ** 2)

    # texture path vs the global-memory caster (T5 image of the same volume): the texture path samples with
    # texel-centre addressing, correct weights and 8-bit fractional weights like a hardware filter (ref
    # raycast.cu:374-433 vs :321-371), so it agrees within a tolerance, not bit for bit
    TEX_MEAN_ABS_DIFF, TEX_MEAN_DIFF = 6.0, 3.0

    def check(self, reduce: bool = True):
        """texture: the timed image against the global-memory caster within the tolerance above; global: bit for
        bit against the serial CPU caster (ref raycast.cu:216-267) up to a 128^2 image (the 512^2 CPU oracle takes
        ~20 s), else against the global caster's own host-side rerun."""
        img = self.image.float()
        if self.method == "texture":
            ref = ops.raycast(self.data, self.region, self.image_dim, method="global").float()
            mad = (img - ref).abs().mean().item()
            md = abs(img.mean().item() - ref.mean().item())
            return {"mean_abs_diff_vs_global": mad, "mean_diff_vs_global": md,
                    "check_passed": mad < self.TEX_MEAN_ABS_DIFF and md < self.TEX_MEAN_DIFF}
        if self.image_dim <= 128 or not self.data.is_cuda:
            ref = ops.raycast(self.data.cpu(), self.region.cpu(), self.image_dim, method="global")
            return {"bit_exact_vs_cpu": bool(torch.equal(self.image.cpu(), ref)),
                    "check_passed": bool(torch.equal(self.image.cpu(), ref))}
        again = ops.raycast(self.data, self.region, self.image_dim, method=self.method)
        return {"deterministic": bool(torch.equal(again, self.image)), "check_passed": bool(torch.equal(again, self.image))}


class Histeq(Workload):
    def __init__(self, ctx, side=4096, **_):
        super().__init__(ctx, {"side": side}, "histeq", "Gpix/s")
        g = torch.Generator().manual_seed(7)
        self.img = torch.randint(0, 200, (side, side), dtype=torch.uint8, generator=g).to(ctx.device)

    def step(self):
        self.out = ops.histeq(self.img)

    def work_per_step(self):
        return float(self.img.numel())

    def check(self, reduce: bool = True):
        """Bit for bit against the serial host oracle (T3; ref 4-histogram-equalization-openmp-pthreads/
        histogram_serial.c:11-42)."""
        ref = ops.histeq(self.img.cpu(), method="serial")
        ok = torch.equal(self.out.cpu(), ref)
        return {"bit_exact_vs_serial": bool(ok), "check_passed": bool(ok)}


class Region2D(Workload):
    """The reference's MPI region-growing app on one device: corner-seeded 4-connected flood fill with
    |a-b| < 2 over pic1.bmp (ref 2-mpi-region-growing/region.c:493-533, 582-604). side > 512 tiles pic1 to
    side x side (longer propagation paths, more tiles); a step regrows from the seeds."""

    def __init__(self, ctx, side=512, **_):
        super().__init__(ctx, {"side": side}, "region2d", "Mpix/s")
        from pathlib import Path

        from ..utils import bmp

        self.assets = Path(__file__).resolve().parents[2] / "assets"
        pic = torch.from_numpy(bmp.read(self.assets / "pic1.bmp").copy())
        reps = max(1, -(-side // pic.shape[0]))
        self.img = pic.repeat(reps, reps)[:side, :side].contiguous().to(ctx.device)
        self.side = side

    def step(self):
        self.region = ops.region2d(self.img)

    def work_per_step(self):
        return float(self.img.numel())

    def scale(self):
        return 1e6

    def check(self, reduce: bool = True):
        """side 512: the output image (pixels of the region zeroed, ref region.c:572-580) equals the reference's
        golden out.bmp (T1, 64,420 region pixels); other sides: the region equals the serial CPU flood fill."""
        from ..utils import bmp

        reg = self.region.cpu() != 0
        if self.side == 512:
            golden = torch.from_numpy(bmp.read(self.assets / "region_pic1_golden.bmp").copy())
            out = self.img.cpu() * (~reg).to(torch.uint8)
            ok = torch.equal(out, golden)
            return {"region_pixels": int(reg.sum()), "golden_pixels": 64420, "matches_golden_bmp": bool(ok),
                    "check_passed": bool(ok)}
        ref = ops.region2d(self.img.cpu()) != 0
        ok = torch.equal(reg, ref)
        return {"region_pixels": int(reg.sum()), "matches_cpu_oracle": bool(ok), "check_passed": bool(ok)}


WORKLOADS = {"sgemm": Sgemm, "reduce": Reduce, "scan": Scan, "stencil": Stencil, "spmv": SpMV,
             "region3d": Region3D, "raycast": Raycast, "histeq": Histeq, "region2d": Region2D}


def build_workload(name: str, ctx: Context, **cfg) -> Workload:
    return WORKLOADS[name](ctx, **cfg)
