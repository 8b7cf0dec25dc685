"""Scan tile-size sweep on 1e9 f32 (rows per lane 8/16, 128-KiB tiles): device time, GB/s (8 B/element), exactness.
Calls pcmx_scan_f32_rows (the per-call tile-shape entry point of libpcmx_hip) through ctypes."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd._native import hip_lib  # noqa: E402
from parallel_c_programs_amd.utils.timing import device_time_ms  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
x = torch.empty(n, device="cuda")
ops.rand_uniform_(x, 7, 0.0, 1.0)
y = torch.empty_like(x)
lib = hip_lib()
lib.pcmx_scan_workspace_bytes.restype = ctypes.c_longlong
ws = torch.empty(lib.pcmx_scan_workspace_bytes(ctypes.c_longlong(n)), dtype=torch.uint8, device="cuda")
ref = torch.cumsum(x[: 1 << 22].double(), 0)
for rows in (8, 16):
    def run():
        rc = lib.pcmx_scan_f32_rows(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_longlong(n), 0,
                                    None, ctypes.c_void_p(ws.data_ptr()), None, rows,
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc

    ms = device_time_ms(run, reps=10, warmup=2)
    err = ((y[: 1 << 22].double() - ref).abs().max() / ref[-1]).item()
    print(f"rows={rows:2d}  {ms:7.3f} ms  {8 * n / ms / 1e6:7.1f} GB/s  rel_err={err:.2e}", flush=True)
