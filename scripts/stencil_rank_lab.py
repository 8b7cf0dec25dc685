"""Stencil rank lab: one rank's compute per distributed step of the 16384^2 bf16 grid at N = 2 / 4 / 8
(an interior rank's slab: 8192 / 4096 / 2048 rows, `fuse` halo rows each side), on one GPU without the halo
exchange, for the launch shapes a step can take:

  full      one launch over all rows (no overlap split)
  split3    interior launch + one launch per edge band (round-2 step)
  split2    interior launch + both edge bands in ONE two-span launch
  split2c   split2 with the edge launch on a side stream, concurrent with the interior kernel
  deep3     the same with m = 3 (3T halo rows: one exchange + one edge launch per 3 steps; time per step)
  deep2     the deep-halo schedule (StencilSlab halo_mult=2): per 2 steps an interior launch + one edge launch over
            the two 2T-row halo-dependent bands, then ONE launch over the own rows; the time is per step (pair / 2)

Every variant is checked bit for bit against `full`. Prints ms per step and GLUP/s per GPU; with the 1-GPU
full-grid time this bounds the strong-scaling efficiency of the compute part (docs/ARCHITECTURE.md, stencil).
Run: python scripts/stencil_rank_lab.py [fuse ...]
Env: STENCIL_LAB_WORLDS=8 (subset of 1,2,4,8), STENCIL_LAB_RPW=0,18 (rows per wave forced on the non-edge launches
as an explicit launch shape of each call, ops.stencil.launch_shape; 0 = production rule; one line per value, all in one
process for an A/B).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd.ops.stencil import launch_shape  # noqa: E402

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
    worlds = [int(w) for w in os.environ.get("STENCIL_LAB_WORLDS", "1,2,4,8").split(",")]
    rpws = [int(r) for r in os.environ.get("STENCIL_LAB_RPW", "0").split(",")]
    for T, world, rpw in [(T, w, r) for T in fuses for w in worlds for r in rpws]:
        shape = launch_shape(0, rpw)

        def step(*a, shape=shape, **kw):  # the non-edge launches take the forced rows per wave
            return ops.stencil5_fused_step_(*a, shape=shape, **kw)

        if True:
            rows = N // world
            row0 = 0 if world == 1 else rows  # rank 1: both neighbours present (interior rank)
            u = (torch.rand(rows + 2 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
            ref, out = u.clone(), u.clone()

            def full():
                step(u, ref, row0, N, halo=T, steps=T)

            def split3():
                step(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T))
                step(u, out, row0, N, halo=T, steps=T, row_range=(0, T))
                step(u, out, row0, N, halo=T, steps=T, row_range=(rows - T, rows))

            def split2():
                step(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T))
                ops.stencil5_fused_spans_(u, out, ((0, T), (rows - T, rows)), row0, N, halo=T, steps=T)

            side = torch.cuda.Stream(dev)

            def split2c():  # the edge launch on a side stream, concurrent with the interior kernel
                main = torch.cuda.current_stream(dev)
                side.wait_stream(main)
                step(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T))
                with torch.cuda.stream(side):
                    ops.stencil5_fused_spans_(u, out, ((0, T), (rows - T, rows)), row0, N, halo=T, steps=T)
                main.wait_stream(side)

            # deep halo (m = 2): a slab with 2T halo rows; step 1 covers local rows [-T, rows + T) (interior launch +
            # edge spans), step 2 the own rows; checked against the same two steps as single full launches
            u2 = (torch.rand(rows + 4 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
            v2, w2, ref2 = u2.clone(), u2.clone(), u2.clone()

            def deep2():
                step(u2, v2, row0, N, halo=2 * T, steps=T, row_range=(T, rows - T))
                ops.stencil5_fused_spans_(u2, v2, ((-T, T), (rows - T, rows + T)), row0, N, halo=2 * T, steps=T)
                step(v2, w2, row0, N, halo=2 * T, steps=T, row_range=(0, rows))

            step(u2, ref2, row0, N, halo=2 * T, steps=T, row_range=(-T, rows + T))
            ref3 = ref2.clone()
            step(ref2, ref3, row0, N, halo=2 * T, steps=T, row_range=(0, rows))

            # deep halo m = 3: 3T halo rows, one exchange + one edge launch per 3 steps
            u3 = (torch.rand(rows + 6 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
            p3, q3, r3 = u3.clone(), u3.clone(), u3.clone()

            def deep3():
                step(u3, p3, row0, N, halo=3 * T, steps=T, row_range=(T, rows - T))
                ops.stencil5_fused_spans_(u3, p3, ((-2 * T, T), (rows - T, rows + 2 * T)), row0, N, halo=3 * T, steps=T)
                step(p3, q3, row0, N, halo=3 * T, steps=T, row_range=(-T, rows + T))
                step(q3, r3, row0, N, halo=3 * T, steps=T, row_range=(0, rows))

            s1, s2, s3 = u3.clone(), u3.clone(), u3.clone()
            step(u3, s1, row0, N, halo=3 * T, steps=T, row_range=(-2 * T, rows + 2 * T))
            step(s1, s2, row0, N, halo=3 * T, steps=T, row_range=(-T, rows + T))
            step(s2, s3, row0, N, halo=3 * T, steps=T, row_range=(0, rows))

            # deep halo m = 4 (generic form of deep2 / deep3)
            M4 = 4
            u4 = (torch.rand(rows + 2 * M4 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
            b4 = [u4.clone() for _ in range(M4 + 1)]

            def deep4():
                e0 = (M4 - 1) * T
                step(b4[0], b4[1], row0, N, halo=M4 * T, steps=T, row_range=(T, rows - T))
                ops.stencil5_fused_spans_(b4[0], b4[1], ((-e0, T), (rows - T, rows + e0)), row0, N, halo=M4 * T,
                                          steps=T)
                for ph in range(1, M4):
                    e = (M4 - 1 - ph) * T
                    step(b4[ph], b4[ph + 1], row0, N, halo=M4 * T, steps=T, row_range=(-e, rows + e))

            c4 = [u4.clone() for _ in range(M4 + 1)]
            for ph in range(M4):
                e = (M4 - 1 - ph) * T
                step(c4[ph], c4[ph + 1], row0, N, halo=M4 * T, steps=T, row_range=(-e, rows + e))

            full()
            res = {}
            for name, fn in (("full", full), ("split3", split3), ("split2", split2), ("split2c", split2c),
                             ("deep2", deep2), ("deep3", deep3), ("deep4", deep4)):
                out.zero_()
                fn()
                torch.cuda.synchronize()
                if name == "deep2":
                    same = torch.equal(w2[2 * T:-2 * T], ref3[2 * T:-2 * T])
                    res[name] = (timed(fn) / 2, same)
                    continue
                if name == "deep4":
                    hh = M4 * T
                    same = torch.equal(b4[M4][hh:-hh], c4[M4][hh:-hh])
                    res[name] = (timed(fn) / M4, same)
                    continue
                if name == "deep3":
                    same = torch.equal(r3[3 * T:-3 * T], s3[3 * T:-3 * T])
                    res[name] = (timed(fn) / 3, same)
                    continue
                same = name == "full" or torch.equal(out[T:-T], ref[T:-T])
                res[name] = (timed(fn), same)
            line = " ".join(f"{k} {ms:.4f} ms {rows * N * T / ms / 1e6:7.0f} GLUP/s{'' if ok else ' MISMATCH'}"
                            for k, (ms, ok) in res.items())
            tag = f" rpw={rpw}" if rpw else ""
            print(f"fuse={T} N={world} rows={rows:5d}{tag}  {line}", flush=True)
            del u, ref, out, u2, v2, w2, ref2, ref3, u3, p3, q3, r3, s1, s2, s3, u4, b4, c4
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
