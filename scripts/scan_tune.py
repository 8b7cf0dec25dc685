"""Scan tile-size sweep on 1e9 f32 (rows per lane 8/16, 128-KiB tiles): device time, GB/s (8 B/element), exactness."""
import sys

import torch

sys.path.insert(0, ".")
from parallel_c_programs_amd import _C, ops  # noqa: E402
from parallel_c_programs_amd.utils.timing import device_time_ms  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
x = torch.empty(n, device="cuda")
ops.rand_uniform_(x, 7, 0.0, 1.0)
y = torch.empty_like(x)
o = torch.ops.pcmx
ref = torch.cumsum(x[: 1 << 22].double(), 0)
for rows in (8, 16):
    _C.scan_set_rows(rows)
    ms = device_time_ms(lambda: o.scan_out(x, y, False, None), reps=10, warmup=2)
    err = ((y[: 1 << 22].double() - ref).abs().max() / ref[-1]).item()
    print(f"rows={rows:2d}  {ms:7.3f} ms  {8 * n / ms / 1e6:7.1f} GB/s  rel_err={err:.2e}", flush=True)
