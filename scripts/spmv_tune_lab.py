"""SpMV tuning lab (one MI355X, 1e8-nnz power-law, packed production kernel): slices x item size x resident
blocks per CU (mode bits 8+), whole product time; every variant checked against the fp64 layout reference.
Run: python scripts/spmv_tune_lab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd.ops.sparse import powerlaw_csr_rows, powerlaw_row_ptr  # noqa: E402


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


dev = torch.device("cuda", 0)
n, nnz = 10_000_000, 100_000_000
rp = powerlaw_row_ptr(n, nnz, 2.5, 1)
m = powerlaw_csr_rows(rp, 0, n, n, 1)
m = ops.CSR(m.row_ptr.to(dev), m.col.to(dev), m.val.to(dev), n)
x = torch.rand(n, device=dev)
for S in (24, 32):
    for item in (512, 1024):
        s = ops.SlicedCSR(m, S, head=0.0625, item_nnz=item)
        ref = s.reference(x)
        for pb in (2, 3, 4, 5):
            y = s.spmv(x, mode=pb << 8).double()
            err = ((y - ref).abs().max() / ref.abs().max()).item()
            ms = timed(lambda: s.spmv(x, mode=pb << 8))
            print(f"slices {S} item {item:4d} blocks/CU {pb}: {ms:.4f} ms {2 * nnz / ms / 1e6:.1f} GFLOP/s err {err:.1e}",
                  flush=True)
        del s
        torch.cuda.empty_cache()
