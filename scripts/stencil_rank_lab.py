"""Stencil rank lab: one rank's compute per distributed step of the 16384^2 bf16 grid at N = 2 / 4 / 8
(an interior rank's slab: 8192 / 4096 / 2048 rows, `fuse` halo rows each side), on one GPU without the halo
exchange, for the launch shapes a step can take:

  full      one launch over all rows (no overlap split)
  split3    interior launch + one launch per edge band (round-2 step)
  split2    interior launch + both edge bands in ONE two-span launch
  split2c   split2 with the edge launch on a side stream, concurrent with the interior kernel (current step)

Every variant is checked bit for bit against `full`. Prints ms per step and GLUP/s per GPU; with the 1-GPU
full-grid time this bounds the strong-scaling efficiency of the compute part (docs/ARCHITECTURE.md, stencil).
Run: python scripts/stencil_rank_lab.py [fuse ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402

N = 16384


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    fuses = [int(a) for a in sys.argv[1:]] or [4, 6, 8]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    for T in fuses:
        for world in (1, 2, 4, 8):
            rows = N // world
            row0 = 0 if world == 1 else rows  # rank 1: both neighbours present (interior rank)
            u = (torch.rand(rows + 2 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
            ref, out = u.clone(), u.clone()

            def full():
                ops.stencil5_fused_step_(u, ref, row0, N, halo=T, steps=T)

            def split3():
                ops.stencil5_fused_step_(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T))
                ops.stencil5_fused_step_(u, out, row0, N, halo=T, steps=T, row_range=(0, T))
                ops.stencil5_fused_step_(u, out, row0, N, halo=T, steps=T, row_range=(rows - T, rows))

            def split2():
                ops.stencil5_fused_step_(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T))
                ops.stencil5_fused_spans_(u, out, ((0, T), (rows - T, rows)), row0, N, halo=T, steps=T)

            side = torch.cuda.Stream(dev)

            def split2c():  # the edge launch on a side stream, concurrent with the interior kernel
                main = torch.cuda.current_stream(dev)
                side.wait_stream(main)
                ops.stencil5_fused_step_(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T))
                with torch.cuda.stream(side):
                    ops.stencil5_fused_spans_(u, out, ((0, T), (rows - T, rows)), row0, N, halo=T, steps=T)
                main.wait_stream(side)

            full()
            res = {}
            for name, fn in (("full", full), ("split3", split3), ("split2", split2), ("split2c", split2c)):
                out.zero_()
                fn()
                torch.cuda.synchronize()
                same = name == "full" or torch.equal(out[T:-T], ref[T:-T])
                res[name] = (timed(fn), same)
            line = " ".join(f"{k} {ms:.4f} ms {rows * N * T / ms / 1e6:7.0f} GLUP/s{'' if ok else ' MISMATCH'}"
                            for k, (ms, ok) in res.items())
            print(f"fuse={T} N={world} rows={rows:5d}  {line}", flush=True)
            del u, ref, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
