"""SpMV row-chunk overlap lab: the 1e8-nnz power-law product cut into C row chunks (one SlicedCSR each); chunk
q's combine (HBM-streaming over its compact partials) runs on a second stream while chunk q + 1's products
(L2-request bound, profiles/r3_spmv/pmc_memory_pipeline.txt) run on the main stream. Compares against the
serial per-chunk order and the one-chunk product. Run: python scripts/spmv_overlap_lab.py [world rank]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd.parallel.dist import Context  # noqa: E402
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
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
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    r = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    dev = torch.device("cuda", 0)
    n, nnz = 10_000_000, 100_000_000
    side = torch.cuda.Stream(device=dev)
    for C in (1, 2, 3, 4, 6, 8):
        d = DistributedSpMV.powerlaw(Context(rank=r, world=W, device=dev), n, nnz, slices=-1, chunks=C)
        xp = torch.rand(d.n_pad, device=dev)
        dsts = [torch.empty(max(1, b - a), device=dev) for a, b, _ in d.parts]
        ref = d.reference_local(xp)
        for pb in (0, 2, 3, 4):
            hi = pb << 8

            def serial():
                for (a, b, part), dst in zip(d.parts, dsts):
                    part.spmv(xp, dst[:b - a], hi)

            def overlap():
                main = torch.cuda.current_stream(dev)
                for (a, b, part), dst in zip(d.parts, dsts):
                    part.spmv(xp, dst[:b - a], hi | 16)
                    ev = torch.cuda.Event()
                    ev.record(main)
                    side.wait_event(ev)
                    with torch.cuda.stream(side):
                        part.spmv(xp, dst[:b - a], 32)
                ev = torch.cuda.Event()
                ev.record(side)
                main.wait_event(ev)

            for name, fn in (("serial", serial), ("overlap", overlap)):
                if C == 1 and name == "overlap":
                    continue
                ms = timed(fn)
                got = torch.cat([dst[:b - a] for (a, b, _), dst in zip(d.parts, dsts)]).double()
                err = ((got - ref).abs().max() / ref.abs().max()).item()
                print(f"N={W} rank {r} slices {d.slices} chunks {C} persist {pb or 'def'} {name:8s} {ms:.4f} ms "
                      f"({2 * d.local_nnz / ms / 1e6:.1f} GFLOP/s) err {err:.1e}", flush=True)
        del d, xp, dsts, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
