"""SpMV host-overhead lab (round 4): is one N = 8 rank's column-split step launch-bound? One rank's products emulated
on one GPU (no exchange), the step's host work without the collectives (4 product launches, 2 combine + fix-up
launches, 2 send-buffer packs): host time per step measured by enqueueing K steps back to back with no sync
(perf_counter) against the device time of the same K steps (events). The two exchange calls a real step adds cost
~13-19 us of host time each (scripts/host_overhead_lab.py, profiles/r2_bench/host_overhead_lab.txt).
Run: python scripts/spmv_host_lab.py [world] [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd.parallel.dist import Context  # noqa: E402
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dev = torch.device("cuda", 0)
    item = int(os.environ.get("SPMV_LAB_ITEM", "512"))
    slices = int(os.environ.get("SPMV_LAB_SLICES", "16"))
    d = DistributedSpMV.powerlaw(Context(rank=0, world=W, device=dev), 10_000_000, 100_000_000, slices=slices, chunks=2,
                                 item_nnz=item, colsplit=True)
    print(f"item_nnz {item}, slices {slices}", flush=True)
    xp = torch.rand(d.n_pad, device=dev)
    out = torch.zeros_like(xp)
    Wd, r = d.ctx.world, d.ctx.rank
    # send lists as the real exchange builds them: per chunk, one ascending subset of the chunk's own rows per peer,
    # as many entries in total as this rank receives (a random graph is symmetric on average)
    packs = []
    for c, (a, b, _) in enumerate(d.parts):
        s0, own = d.seg[c * Wd + r], b - a
        k = max(1, d.ghost_len[c] // (Wd - 1))
        packs.append(torch.cat([s0 + torch.sort(torch.randperm(own, device=dev)[:min(k, own)]).values
                                for _ in range(Wd - 1)]))
    packs32 = [p.to(torch.int32) for p in packs]
    bufs = [torch.empty(p.numel(), device=dev) for p in packs]
    from parallel_c_programs_amd.ops.vector import gather_
    print(f"send entries per step {sum(p.numel() for p in packs)}, ghosts received {d.n_ghost}", flush=True)

    def step(pack="gather"):
        for c, (a, b, part) in enumerate(d.parts):
            if b > a:
                part.product_phase(xp, 0, c)
        for c, (a, b, part) in enumerate(d.parts):
            s0 = d.seg[c * Wd + r]
            if b > a:
                part.product_phase(xp, 1, c, out[s0:s0 + (b - a)])
            if pack == "index_select":
                torch.index_select(out, 0, packs[c], out=bufs[c])
            elif pack:
                gather_(out, packs32[c], bufs[c])

    side = torch.cuda.Stream(device=dev)
    ev = torch.cuda.Event()

    def step_overlap():
        """chunk 0's combine + fix-up + pack on a side stream, beside chunk 1's phase-1 products"""
        main = torch.cuda.current_stream(dev)
        for c, (a, b, part) in enumerate(d.parts):
            if b > a:
                part.product_phase(xp, 0, c)
        for c, (a, b, part) in enumerate(d.parts):
            s0 = d.seg[c * Wd + r]
            half = part.n_slices // 16
            part.spmv(xp, mode=16, phases=(half, half))
            if c == 0:
                ev.record(main)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    part.spmv(xp, out[s0:s0 + (b - a)], mode=32)
                    gather_(out, packs32[c], bufs[c])
            else:
                part.spmv(xp, out[s0:s0 + (b - a)], mode=32)
                gather_(out, packs32[c], bufs[c])
        main.wait_stream(side)

    for _ in range(10):
        step()
        step_overlap()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    t1 = time.perf_counter()
    e1.record()
    e1.synchronize()
    host = (t1 - t0) / reps * 1e3
    devt = e0.elapsed_time(e1) / reps
    e0.record()
    for _ in range(reps):
        step(False)
    e1.record()
    e1.synchronize()
    print(f"N={W} products only (no packs): device {e0.elapsed_time(e1) / reps:.4f} ms/step", flush=True)
    e0.record()
    for _ in range(reps):
        step("index_select")
    e1.record()
    e1.synchronize()
    print(f"N={W} with torch.index_select (int64) packs: device {e0.elapsed_time(e1) / reps:.4f} ms/step", flush=True)
    e0.record()
    for _ in range(reps):
        step_overlap()
    e1.record()
    e1.synchronize()
    print(f"N={W} chunk 0's combine + pack on a side stream beside chunk 1's products: device "
          f"{e0.elapsed_time(e1) / reps:.4f} ms/step", flush=True)
    for pb in (1, 2, 3, 4, 6, 8):  # resident sliced blocks per CU of the product launches (kernel mode bits 8-15)
        def products_pb():
            for ph in (0, 1):
                for c, (a, b, part) in enumerate(d.parts):
                    half = part.n_slices // 16
                    part.spmv(xp, mode=16 | (pb << 8), phases=(ph * half, half))
        for _ in range(3):
            products_pb()
        e0.record()
        for _ in range(reps):
            products_pb()
        e1.record()
        e1.synchronize()
        print(f"N={W} the 4 product launches alone, {pb} resident blocks per CU: {e0.elapsed_time(e1) / reps:.4f} ms/step",
              flush=True)
    print(f"N={W} rank 0 column-split step: host enqueue {host:.4f} ms/step, device {devt:.4f} ms/step "
          f"({'launch-bound' if host > devt else 'device-bound'}; + ~0.03 ms of host time for the 2 exchange calls)",
          flush=True)


if __name__ == "__main__":
    main()
