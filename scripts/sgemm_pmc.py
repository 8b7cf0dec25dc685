"""Run one SGEMM variant and torch.matmul a few times (for rocprofv3 --pmc)."""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402
n = int(sys.argv[1]); v = int(sys.argv[2])
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
for _ in range(3):
    ops.sgemm(a, b, variant=v)
    a @ b
torch.cuda.synchronize()
