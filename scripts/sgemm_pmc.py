"""Run one SGEMM variant and torch.matmul a few times (for rocprofv3 --pmc). Production variants (0, 1, 16) run
from libpcmx_hip; any other number runs the lab build (scripts/sgemm_lab.hip)."""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402
n = int(sys.argv[1]); v = int(sys.argv[2])
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
sys.path.insert(0, str(Path(__file__).resolve().parent))
import _lab  # noqa: E402

for _ in range(3):
    ops.sgemm(a, b, variant=v) if v in (0, 1, 16) else _lab.sgemm(a, b, v)
    a @ b
torch.cuda.synchronize()
