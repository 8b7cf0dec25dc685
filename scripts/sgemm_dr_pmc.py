"""Runs SGEMM kernels a few times each for rocprofv3 --pmc: production ops.sgemm_out ("prod"), direct-register lab
variants (numbers, scripts/sgemm_dr_lab.hip) and torch.matmul (hipBLASLt). usage: sgemm_dr_pmc.py N prod,34,..."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402
sys.path.insert(0, str(Path(__file__).resolve().parent))
import _lab  # noqa: E402

n = int(sys.argv[1])
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
c = torch.empty(n, n, device="cuda")
for v in sys.argv[2].split(","):
    for _ in range(4):
        if v == "prod":
            ops.sgemm_out(a, b, c)
        elif v == "torch":
            torch.matmul(a, b, out=c)
        else:
            _lab.sgemm_dr(a, b, int(v), c)
    torch.cuda.synchronize()
