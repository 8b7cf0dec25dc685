"""SGEMM lab: fixed (K-independent) cost per launch — prologue, epilogue, tail, launch — from a linear fit of
time vs K at M = N = 8192 (production variant 16, direct-register lab variants 30/34/35, hipBLASLt)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import _lab  # noqa: E402
from parallel_c_programs_amd import ops  # noqa: E402


def t_ms(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


n = 8192
Ks = [1024, 2048, 4096, 8192]
res = {}
for rnd in range(3):
    for k in Ks:
        a = torch.rand(n, k, device="cuda") * 2 - 1
        b = torch.rand(k, n, device="cuda") * 2 - 1
        c = torch.empty(n, n, device="cuda")
        for name, fn in (("v16", lambda: ops.sgemm_out(a, b, c)), ("dr30", lambda: _lab.sgemm_dr(a, b, 30, c)),
                         ("drp34", lambda: _lab.sgemm_dr(a, b, 34, c)), ("drp35_nostore", lambda: _lab.sgemm_dr(a, b, 35, c)),
                         ("torch", lambda: torch.matmul(a, b, out=c))):
            res.setdefault((name, k), []).append(t_ms(fn))
for name in ("v16", "dr30", "drp34", "drp35_nostore", "torch"):
    pts = [(k, min(res[(name, k)])) for k in Ks]
    nk = len(pts)
    mk = sum(k for k, _ in pts) / nk
    mt = sum(t for _, t in pts) / nk
    slope = sum((k - mk) * (t - mt) for k, t in pts) / sum((k - mk) ** 2 for k, _ in pts)
    icpt = mt - slope * mk
    print(json.dumps({"impl": name, "ms": {k: round(t, 4) for k, t in pts}, "fixed_ms": round(icpt, 4),
                      "ms_per_1k_k": round(slope * 1024, 4),
                      "asymptotic_tflops": round(2.0 * n * n * 1024 / (slope * 1024) / 1e9, 1)}))
