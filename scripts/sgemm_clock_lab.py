"""Clock under sustained MFMA load (the fp32-via-bf16x6 GEMM runs 265-267 TF in 10-call bursts and
244-258 sustained). Runs 40 back-to-back 8192^3 GEMMs of each kernel (native f32 MFMA, then x6 on the bf16 matrix
cores), meant to run under `rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES`; scripts/clock_summary.py
then divides each dispatch's GRBM_GUI_ACTIVE by its duration (cycles per ns ~ the engine clock, up to a constant
factor of the counter's aggregation) and compares the first and last calls of each run.
usage: python scripts/sgemm_clock_lab.py [calls]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 40
n = 8192
a = torch.empty(n, n, device="cuda")
b = torch.empty(n, n, device="cuda")
c = torch.empty(n, n, device="cuda")
ops.rand_uniform_(a, 1)
ops.rand_uniform_(b, 2)
for variant in (-1, 20):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(calls):
        ops.sgemm_out(a, b, c, variant=variant)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / calls
    print(f"variant {variant}: {calls} calls, {ms:.3f} ms/call, {2 * n ** 3 / ms / 1e9:.1f} TFLOPS", flush=True)
