"""Which torch call reaches hipSPARSE fastest for the 1e8-nnz power-law CSR (the bench's vendor bar)? Times
torch.mv / @ / torch.sparse.mm with int32 and int64 indices (HIP events, median of 5 after 2 warm-ups)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd.parallel.dist import Context  # noqa: E402
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV  # noqa: E402

n, nnz = (int(float(a)) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (1e7, 1e8)))
d = DistributedSpMV.powerlaw(Context(device=torch.device("cuda")), n, nnz, slices=0, keep_plain=True)
m = d.plain
x = torch.rand(m.n_cols, device="cuda")
ref = None


def t(fn):
    for _ in range(2):
        y = fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        y = fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[2], y


for idx in (torch.int32, torch.int64):
    A = torch.sparse_csr_tensor(m.row_ptr.to(idx), m.col.to(idx), m.val, size=(m.n_rows, m.n_cols))
    for name, fn in (("mv", lambda: torch.mv(A, x)), ("matmul", lambda: A @ x),
                     ("sparse.mm", lambda: torch.sparse.mm(A, x.unsqueeze(1)).squeeze(1))):
        try:
            ms, y = t(fn)
            ref = y if ref is None else ref
            print(json.dumps({"index": str(idx), "call": name, "ms": round(ms, 3), "gflops": round(2 * m.nnz / ms / 1e6, 2),
                              "max_abs_diff_vs_first": (y - ref).abs().max().item()}), flush=True)
        except Exception as ex:  # noqa: BLE001
            print(json.dumps({"index": str(idx), "call": name, "error": f"{type(ex).__name__}: {ex}"[:200]}), flush=True)
