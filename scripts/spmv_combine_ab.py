"""SpMV combine A/B (one MI355X, 1e8-nnz power-law, production sliced layout): the ballot-rank combine (mode bit 6)
against the byte-packed-scan combine (default), each timed ALONE on the partials one product wrote (mode bit 5 =
combine + fix-up only), plus the whole product both ways; the two y must be bit-identical.
Run: python scripts/spmv_combine_ab.py [slices ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd.ops.sparse import powerlaw_csr_rows, powerlaw_row_ptr  # noqa: E402


def timed(fn, reps=30):
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
for S in [int(a) for a in sys.argv[1:]] or [24, 16]:
    s = ops.SlicedCSR(m, S, head=0.0625, item_nnz=1024)
    ref = s.reference(x)
    y_scan = s.spmv(x).clone()
    y_ballot = s.spmv(x, mode=64).clone()
    same = torch.equal(y_scan, y_ballot)
    err = ((y_scan.double() - ref).abs().max() / ref.abs().max()).item()
    s.spmv(x, mode=16)  # partials for the combine-only timings
    t_scan = timed(lambda: s.spmv(x, mode=32))
    t_ballot = timed(lambda: s.spmv(x, mode=32 | 64))
    p_scan = timed(lambda: s.spmv(x))
    p_ballot = timed(lambda: s.spmv(x, mode=64))
    print(f"slices {S}: partials {s.partials}  combine+fixup ballot {t_ballot * 1e3:.1f} us  scan {t_scan * 1e3:.1f} us"
          f"  | product ballot {p_ballot:.4f} ms ({2 * nnz / p_ballot / 1e6:.1f} GFLOP/s)  scan {p_scan:.4f} ms"
          f" ({2 * nnz / p_scan / 1e6:.1f} GFLOP/s)  bit-identical {same}  err {err:.1e}", flush=True)
    del s
    torch.cuda.empty_cache()
