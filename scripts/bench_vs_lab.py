"""Bench vs lab, in ONE process on one MI355X (round-5 VERDICT item 4): for the stencil, reduce and SpMV sections, the
bench's own timing (workloads.<Section>.step through utils.harness.timed: W warm-ups, K steps between barrier + sync,
per-step hipEvents) against the lab's timing (back-to-back launches of the same kernel on the same data between two
events), each measured
  cold  right after the section is set up (what the bench does),
  hot   right after 25 back-to-back fp32-via-bf16x6 SGEMMs (the bench runs its sections after the SGEMM section;
        the x6 kernel holds the chip at a power-limited clock),
  again after an idle second (clock recovered),
so the cause of a bench-vs-lab gap can be told apart: harness (bench vs lab in the same state), clock (hot vs
again), or data / shape. Stencil extras: the full launch vs the split2 interior + two-span edge launch at 16384 rows
(interleaved rounds), and the random bench grid vs the round-4 hot-square grid.
usage: python scripts/bench_vs_lab.py [K] [W]"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd.models import workloads as W  # noqa: E402
from parallel_c_programs_amd.parallel import init  # noqa: E402
from parallel_c_programs_amd.utils.harness import timed  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
WU = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ctx = init()
dev = ctx.device


def lab(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def bench(fn):
    ms = []
    t = timed(ctx, fn, K, WU, ms)
    return 1e3 * t / K, statistics.median(ms)


g = W.Sgemm(ctx, n=8192, variant=20)


def heat():
    for _ in range(25):
        g.step()
    torch.cuda.synchronize()


def report():
    for state in ("cold", "hot", "again"):
        if state == "hot":
            heat()
        elif state == "again":
            time.sleep(1.0)
        yield state


def line(sec, state, kind, ms, work, unit):
    print(f"{sec:8s} {state:5s} {kind:18s} {ms:.4f} ms  {work / ms / 1e6:9.1f} {unit}", flush=True)


# ---- stencil 16384^2 bf16, T = 8 (the N = 1 bench shape)
s = W.Stencil(ctx, n=16384)
T, n = s.slab.fuse, s.slab.n
cells = n * n * T
for state in report():
    wall, med = bench(s.step)
    line("stencil", state, "bench wall", wall, cells, "GLUP/s")
    line("stencil", state, "bench device med", med, cells, "GLUP/s")
    u, v = s.slab.u, s.slab.v
    line("stencil", state, "lab full", lab(lambda: ops.stencil5_fused_step_(u, v, 0, n, halo=T, steps=T)), cells,
         "GLUP/s")
# full vs split2 at 16384 rows (the N = 1 question: does the two-launch form beat the single launch?), interleaved
u, v = s.slab.u, s.slab.v
full_fn = lambda: ops.stencil5_fused_step_(u, v, 0, n, halo=T, steps=T)  # noqa: E731


def split2():
    ops.stencil5_fused_step_(u, v, 0, n, halo=T, steps=T, row_range=(T, n - T))
    ops.stencil5_fused_spans_(u, v, ((0, T), (n - T, n)), 0, n, halo=T, steps=T)


ref = v.clone()
full_fn()
a = v.clone()
split2()
same = torch.equal(a, v)
rounds = {"full": [], "split2": []}
for _ in range(6):
    rounds["full"].append(lab(full_fn, 30))
    rounds["split2"].append(lab(split2, 30))
for k, ts in rounds.items():
    print(f"stencil  16384 rows T={T} {k:6s} rounds " + " ".join(f"{t:.4f}" for t in ts) +
          f"  median {statistics.median(ts):.4f} ms" + ("" if same else "  MISMATCH"), flush=True)
# data: random bench grid vs the round-4 hot-square grid
hot = W.Stencil(ctx, n=16384, pattern="hot")
hu, hv = hot.slab.u, hot.slab.v
for _ in range(2):
    line("stencil", "-", "lab full random", lab(full_fn), cells, "GLUP/s")
    line("stencil", "-", "lab full hot-grid",
         lab(lambda: ops.stencil5_fused_step_(hu, hv, 0, n, halo=T, steps=T)), cells, "GLUP/s")
del s, hot, u, v, hu, hv, ref, a
torch.cuda.empty_cache()

# ---- reduce 1e9 f32
r = W.Reduce(ctx, n=10**9)
nbytes = 4 * r.x.numel()
for state in report():
    wall, med = bench(r.step)
    line("reduce", state, "bench wall", wall, nbytes, "GB/s")
    line("reduce", state, "bench device med", med, nbytes, "GB/s")
    line("reduce", state, "lab ops.reduce", lab(lambda: ops.reduce(r.x, "sum")), nbytes, "GB/s")
del r
torch.cuda.empty_cache()

# ---- SpMV 1e8 nnz power-law (one rank, one chunk: the bench step is exactly one sliced product)
sp = W.SpMV(ctx)
(_, _, part), = sp.d.parts
y = torch.empty(part.n_rows, device=dev)
flops = 2.0 * sp.d.local_nnz
for state in report():
    wall, med = bench(sp.step)
    line("spmv", state, "bench wall", wall, flops, "GFLOP/s")
    line("spmv", state, "bench device med", med, flops, "GFLOP/s")
    line("spmv", state, "lab part.spmv", lab(lambda: part.spmv(sp.xp, y)), flops, "GFLOP/s")
