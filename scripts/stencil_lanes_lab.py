"""Stencil lanes lab: 8 vs 4 columns per lane (csrc/kernels/stencil.hip Geo, explicit launch shapes) for the fused
v2 kernel, per slab height (one rank's interior slab at N = 8 / 4 / 2 / 1 of the 16384^2 grid) and rows per wave.
Every configuration is checked bit for bit against the production launch; prints ms and GLUP/s of the full-slab
launch and of the distributed step shape (interior launch + one two-span edge launch).
With "edge" as the first argument it sweeps the EDGE launch shape instead (the two T-row halo bands of a
distributed step) with the interior launch at the production rule.
usage: stencil_lanes_lab.py [T,...] [rows,...] [reps]    |    stencil_lanes_lab.py edge [T,...] [rows,...] [reps]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd.ops.stencil import launch_shape  # noqa: E402

N = 16384


def timed(fn, reps):
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


def edge_sweep(argv):
    fuses = [int(a) for a in argv[0].split(",")] if argv else [4, 6, 8]
    heights = [int(a) for a in argv[1].split(",")] if len(argv) > 1 else [2048, 4096]
    reps = int(argv[2]) if len(argv) > 2 else 40
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    for T in fuses:
        for rows in heights:
            u = (torch.rand(rows + 2 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
            ref, out = u.clone(), u.clone()
            ops.stencil5_fused_step_(u, ref, rows, N, halo=T, steps=T)
            torch.cuda.synchronize()
            for cpl, rpw in ((0, 0), (8, 16), (8, 4), (8, 2), (4, 16), (4, 4), (4, 2)):
                es = launch_shape(cpl, rpw)

                def edges():
                    ops.stencil5_fused_spans_(u, out, ((0, T), (rows - T, rows)), rows, N, halo=T, steps=T, shape=es)

                def split2():
                    ops.stencil5_fused_step_(u, out, rows, N, halo=T, steps=T, row_range=(T, rows - T))
                    edges()

                out.zero_()
                split2()
                torch.cuda.synchronize()
                ok = torch.equal(out[T:-T], ref[T:-T])
                te, ts = timed(edges, reps), timed(split2, reps)
                print(f"T={T} rows={rows:5d} edge cpl={cpl} rpw={rpw:2d} (0 = production)  edge launch {te:.4f} ms"
                      f"  split2 {ts:.4f} ms {rows * N * T / 1e6 / ts:6.0f} GLUP/s{'' if ok else ' MISMATCH'}", flush=True)
            del u, ref, out
            torch.cuda.empty_cache()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "edge":
        return edge_sweep(sys.argv[2:])
    fuses = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else [4, 6, 8]
    heights = [int(a) for a in sys.argv[2].split(",")] if len(sys.argv) > 2 else [2048, 4096, 8192, 16384]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    for T in fuses:
        for rows in heights:
            row0 = 0 if rows == N else rows  # an interior rank (both neighbours) unless the whole grid
            u = (torch.rand(rows + 2 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
            ref, out = u.clone(), u.clone()
            ops.stencil5_fused_step_(u, ref, row0, N, halo=T, steps=T)
            torch.cuda.synchronize()
            for cpl in (8, 4):
                for rpw in (16, 18, 24, 32, 64):
                    fs = launch_shape(cpl, rpw)

                    def full():
                        ops.stencil5_fused_step_(u, out, row0, N, halo=T, steps=T, shape=fs)

                    def split2():
                        ops.stencil5_fused_step_(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T), shape=fs)
                        ops.stencil5_fused_spans_(u, out, ((0, T), (rows - T, rows)), row0, N, halo=T, steps=T)

                    out.zero_()
                    full()
                    torch.cuda.synchronize()
                    ok_full = torch.equal(out[T:-T], ref[T:-T])
                    out.zero_()
                    split2()
                    torch.cuda.synchronize()
                    ok_split = torch.equal(out[T:-T], ref[T:-T])
                    tf, ts = timed(full, reps), timed(split2, reps)
                    glup = rows * N * T / 1e6
                    print(f"T={T} rows={rows:5d} cpl={cpl} rpw={rpw:2d}  full {tf:.4f} ms {glup / tf:6.0f} GLUP/s"
                          f"{'' if ok_full else ' MISMATCH'}  split2 {ts:.4f} ms {glup / ts:6.0f} GLUP/s"
                          f"{'' if ok_split else ' MISMATCH'}", flush=True)
            del u, ref, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
