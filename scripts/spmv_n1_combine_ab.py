"""SpMV at N = 1 (the bench's 1e8-nnz power-law step): the fused combine (combine + split-row fix-up in one launch,
SlicedCSR.fused_combine, round 5) against the two-launch combine + fix-up, interleaved A/B rounds in one process,
bit-identity checked. Run: python scripts/spmv_n1_combine_ab.py [rounds]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd.models import workloads as W  # noqa: E402
from parallel_c_programs_amd.ops.sparse import SlicedCSR  # noqa: E402
from parallel_c_programs_amd.parallel.dist import Context  # noqa: E402


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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ctx = Context(rank=0, world=1, device=torch.device("cuda", 0))
    sp = W.SpMV(ctx)
    parts = [p for _, _, p in sp.d.parts if isinstance(p, SlicedCSR)]

    def set_fused(on):  # an INSTANCE attribute (SlicedCSR.__init__ sets it per matrix)
        for p in parts:
            p.fused_combine = on

    outs = {}
    for fused in (True, False):
        set_fused(fused)
        sp.step()
        torch.cuda.synchronize()
        outs[fused] = sp.y.clone()
    same = torch.equal(outs[True], outs[False])
    print(f"bit-identical fused vs two-launch: {same}", flush=True)
    for r in range(rounds):
        line = []
        for fused in ((True, False) if r % 2 == 0 else (False, True)):
            set_fused(fused)
            ms = timed(sp.step)
            line.append(f"{'fused' if fused else 'two-launch'} {ms:.4f} ms ({2 * sp.d.local_nnz / ms / 1e6:.1f} GFLOP/s)")
        print(f"round {r}: " + "  ".join(line), flush=True)


if __name__ == "__main__":
    main()
