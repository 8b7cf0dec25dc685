"""Interleaved A/B: direct-register lab SGEMM variants (scripts/sgemm_dr_lab.hip) vs the production kernel
(ops.sgemm) vs hipBLASLt (torch.matmul), each timed like bench.py (W warm-up calls, then K calls between events).
usage: sgemm_dr_ab.py N v1,v2,... [rounds] [K]"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402
sys.path.insert(0, str(Path(__file__).resolve().parent))
import _lab  # noqa: E402


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


n = int(sys.argv[1])
variants = [int(v) for v in sys.argv[2].split(",") if v]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
K = int(sys.argv[4]) if len(sys.argv) > 4 else 10
torch.manual_seed(0)
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
c = torch.empty(n, n, device="cuda")
rows = torch.arange(0, n, 37, device="cuda")
ref = a[rows].double() @ b.double()
flop = 2.0 * n ** 3
for v in variants:
    c.zero_()
    _lab.sgemm_dr(a, b, v, c)
    torch.cuda.synchronize()
    err = ((c[rows].double() - ref).abs().max() / ref.abs().max()).item()
    print(json.dumps({"variant": v, "n": n, "max_rel_err_vs_fp64": err}), flush=True)
res = {}
for rnd in range(rounds):
    res.setdefault("prod", []).append(t_ms(lambda: ops.sgemm_out(a, b, c), K))
    for v in variants:
        res.setdefault(f"v{v}", []).append(t_ms(lambda: _lab.sgemm_dr(a, b, v, c), K))
    res.setdefault("hipblaslt", []).append(t_ms(lambda: torch.matmul(a, b, out=c), K))
for k, v in res.items():
    print(json.dumps({"cfg": k, "n": n, "ms_all": [round(x, 4) for x in v], "best_tflops": round(flop / min(v) / 1e9, 2),
                      "median_tflops": round(flop / sorted(v)[len(v) // 2] / 1e9, 2)}), flush=True)
