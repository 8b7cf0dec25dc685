"""Stencil LDS-DMA lab (round 4): the fused stencil's prefetch ring with register loads (production) against the
LDS-DMA ring (`buffer_load_dwordx4 ... lds`, exact hand-counted vmcnt; pcmx_stencil_lab_set(3, 0, 1)) for 8-column
lanes, one fused launch over a ROWS x 16384 bf16 slab, alternating A/B in one process, every DMA result checked bit
for bit against the production launch.
usage: stencil_dma_lab.py [T,...] [rows,...] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd._native import hip_lib  # noqa: E402

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


def main():
    fuses = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else [8, 6]
    heights = [int(a) for a in sys.argv[2].split(",")] if len(sys.argv) > 2 else [16384, 8192]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    lib = hip_lib()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    try:
        for T in fuses:
            for rows in heights:
                u = (torch.rand(rows + 2 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
                ref, out = u.clone(), u.clone()
                assert lib.pcmx_stencil_lab_set(0, 8, 0) == 0  # 8-column lanes, production rows per wave
                assert lib.pcmx_stencil_lab_set(3, 0, 0) == 0
                ops.stencil5_fused_step_(u, ref, rows, N, halo=T, steps=T)
                assert lib.pcmx_stencil_lab_set(3, 0, 1) == 0
                out.zero_()
                ops.stencil5_fused_step_(u, out, rows, N, halo=T, steps=T)
                torch.cuda.synchronize()
                ok = torch.equal(out[T:-T], ref[T:-T])
                res = {0: [], 1: []}
                for _ in range(3):
                    for dma in (0, 1):
                        assert lib.pcmx_stencil_lab_set(3, 0, dma) == 0
                        res[dma].append(timed(lambda: ops.stencil5_fused_step_(u, out, rows, N, halo=T, steps=T), reps))
                a, b = min(res[0]), min(res[1])
                print(f"T={T} rows={rows:5d} cpl=8  registers {a:.4f} ms {rows * N * T / a / 1e6:6.0f} GLUP/s   "
                      f"LDS-DMA {b:.4f} ms {rows * N * T / b / 1e6:6.0f} GLUP/s  ({(a / b - 1) * 100:+.1f}%)"
                      f"{'' if ok else '  MISMATCH'}", flush=True)
                del u, ref, out
                torch.cuda.empty_cache()
    finally:
        lib.pcmx_stencil_lab_set(0, 0, 0), lib.pcmx_stencil_lab_set(3, 0, 0)


if __name__ == "__main__":
    main()
