"""fp32 GEMM on the bf16 matrix cores (variant 20, csrc/kernels/sgemm_x6.hip) vs the native f32-MFMA kernel
(variant 17) vs hipBLASLt (torch.matmul): fp64 error on several shapes / operand ranges, then interleaved timing
like bench.py (W warm-up calls, K calls between events).
usage: sgemm_x6_ab.py [N] [rounds] [K] [x6 schedule variants, e.g. 0,1,2]"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd._native import hip_lib  # noqa: E402
import ctypes  # noqa: E402


def x6(a, b, c, v):
    """variant knob of pcmx_sgemm_f32_x6_variant (0 = production schedule)"""
    m, k = a.shape
    rc = hip_lib().pcmx_sgemm_f32_x6_variant(
        ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(c.data_ptr()), m, b.shape[1], k,
        a.stride(0), b.stride(0), c.stride(0), ctypes.c_float(1.0), ctypes.c_float(0.0), v,
        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc


def t_ms(fn, k=10, w=3):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(k):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / k


def err(c, a, b, rows):
    ref = a[rows].double() @ b.double()
    return ((c[rows].double() - ref).abs().max() / ref.abs().max()).item()


n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
torch.manual_seed(0)
for (m, nn, k, lo) in [(256, 256, 32, 0.0), (512, 768, 96, -1.0), (1024, 1024, 4096, -1.0), (2048, 512, 8192, 0.0)]:
    a = torch.rand(m, k, device="cuda") * (1 - lo) + lo
    b = torch.rand(k, nn, device="cuda") * (1 - lo) + lo
    rows = torch.arange(0, m, 7, device="cuda")
    out = {"shape": [m, nn, k], "range": [lo, 1.0]}
    for v in (17, 20):
        try:
            out[f"v{v}_err"] = err(ops.sgemm(a, b, v), a, b, rows)
        except RuntimeError as e:
            out[f"v{v}_err"] = str(e)[:80]
    out["hipblaslt_err"] = err(a @ b, a, b, rows)
    print(json.dumps(out), flush=True)

a = torch.rand(n, n, device="cuda")
b = torch.rand(n, n, device="cuda")
c = torch.empty(n, n, device="cuda")
rows = torch.arange(0, n, max(1, n // 8), device="cuda")
xv = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0]
for v in (17, 20):
    ops.sgemm_out(a, b, c, variant=v)
    print(json.dumps({"variant": v, "n": n, "max_rel_err_vs_fp64": err(c, a, b, rows)}), flush=True)
for v in xv:
    c.zero_()
    x6(a, b, c, v)
    print(json.dumps({"x6_schedule": v, "n": n, "max_rel_err_vs_fp64": err(c, a, b, rows)}), flush=True)
flop = 2.0 * n ** 3
ah, bh, ch = a.bfloat16(), b.bfloat16(), torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
res = {}
for _ in range(rounds):
    res.setdefault("v17_native_f32", []).append(t_ms(lambda: ops.sgemm_out(a, b, c, variant=17), K))
    for v in xv:
        res.setdefault(f"x6_sched{v}", []).append(t_ms(lambda: x6(a, b, c, v), K))
    res.setdefault("hipblaslt", []).append(t_ms(lambda: torch.matmul(a, b, out=c), K))
    # calibration: the vendor's plain bf16 GEMM rate on this box (x6 does 6x its MFMA work per fp32 GEMM)
    res.setdefault("hipblaslt_bf16_x6_equiv", []).append(6 * t_ms(lambda: torch.matmul(ah, bh, out=ch), K))
for k_, v in res.items():
    print(json.dumps({"cfg": k_, "n": n, "ms_all": [round(x, 4) for x in v], "best_tflops": round(flop / min(v) / 1e9, 2),
                      "median_tflops": round(flop / sorted(v)[len(v) // 2] / 1e9, 2)}), flush=True)
