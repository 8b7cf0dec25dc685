"""Stencil rows-per-wave lab (round 4): rows per wave is a launch parameter of the fused kernel (RowSpans.rpw), so the
grid can be sized to whole residency rounds of the chip. Sweeps rows per wave x columns per lane x prefetch depth for
one fused launch over a slab of `rows` x 16384 bf16 (halo T), checks every result bit for bit against the production
launch and prints ms, GLUP/s and the grid (workgroups, and workgroups per residency round at the kernel's occupancy).
usage: stencil_rpw_lab.py T rows cpl[,cpl] rpw[,rpw...] [ahead[,ahead]] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd.ops.stencil import launch_shape  # noqa: E402

N = 16384
# VGPRs of stencil5xT2_kernel<T, ahead, 1, cpl> (hipcc -S, csrc/kernels/stencil.hip) -> waves per SIMD = 512 // VGPRs
VGPRS = {(8, 3, 8): 222, (8, 6, 8): 234, (8, 9, 8): 246, (8, 3, 4): 112, (8, 6, 4): 118, (8, 9, 4): 124,
         (6, 3, 8): 174, (6, 6, 8): 186, (6, 9, 8): 198, (6, 3, 4): 88, (6, 6, 4): 94, (6, 9, 4): 100,
         (4, 3, 8): 126, (4, 6, 8): 138, (4, 9, 8): 150, (4, 3, 4): 64, (4, 6, 4): 70, (4, 9, 4): 76}


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


def strips(cpl, T):
    L = (T + cpl - 1) // cpl
    out = (64 - 2 * L) * cpl
    return 1 if N <= 64 * cpl else 1 + (N - 64 * cpl + out - 1) // out


def main():
    T, rows = int(sys.argv[1]), int(sys.argv[2])
    cpls = [int(a) for a in sys.argv[3].split(",")]
    rpws = [int(a) for a in sys.argv[4].split(",")]
    aheads = [int(a) for a in sys.argv[5].split(",")] if len(sys.argv) > 5 else [0]
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 30
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    u = (torch.rand(rows + 2 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
    ref, out = u.clone(), u.clone()
    fn_ref = lambda: ops.stencil5_fused_step_(u, ref, rows, N, halo=T, steps=T)  # noqa: E731
    fn_ref()
    torch.cuda.synchronize()
    t_prod = timed(fn_ref, reps)
    print(f"T={T} rows={rows} production {t_prod:.4f} ms {rows * N * T / 1e6 / t_prod:6.0f} GLUP/s", flush=True)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    if True:
        for cpl in cpls:
            for ahead in aheads:
                for rpw in rpws:
                    sh = launch_shape(cpl, rpw, ahead)
                    fn = lambda: ops.stencil5_fused_step_(u, out, rows, N, halo=T, steps=T, shape=sh)  # noqa: E731
                    out.zero_()
                    fn()
                    torch.cuda.synchronize()
                    ok = torch.equal(out[T:-T], ref[T:-T])
                    t = timed(fn, reps)
                    ka = ahead or ((9 if T >= 6 and rpw >= 64 else 3 if rpw <= 4 or 16 < rpw <= 20 else 6))
                    wps = 512 // VGPRS.get((T, ka, cpl), 512)
                    wgs = strips(cpl, T) * -(-rows // (4 * rpw))
                    rounds = wgs / (cus * wps)
                    print(f"T={T} rows={rows} cpl={cpl} ahead={ka} rpw={rpw:3d}  {t:.4f} ms "
                          f"{rows * N * T / 1e6 / t:6.0f} GLUP/s  wgs={wgs} waves/SIMD={wps} rounds={rounds:.2f}"
                          f"{'' if ok else ' MISMATCH'}", flush=True)


if __name__ == "__main__":
    main()
