"""Times the bench's N = 1 SpMV step (W.SpMV(), 1e8 nnz) with whichever package is first on sys.path (an A/B of two
builds in separate processes on one box): python scripts/spmv_step_time.py [package_root] [rounds]"""
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.abspath(root))
import torch  # noqa: E402

from parallel_c_programs_amd.models import workloads as W  # noqa: E402
from parallel_c_programs_amd.parallel.dist import Context  # noqa: E402

sp = W.SpMV(Context(rank=0, world=1, device=torch.device("cuda", 0)))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    for _ in range(5):
        sp.step()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(50):
        sp.step()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 50
    print(f"{root}: round {r} {ms:.4f} ms {2 * sp.d.local_nnz / ms / 1e6:.1f} GFLOP/s", flush=True)
