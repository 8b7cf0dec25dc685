"""Interleaved A/B of the production SGEMM (libpcmx_hip, variant 16) against lab variants and hipBLASLt.
usage: python scripts/sgemm_ab_prod.py N lab_variants(comma) [rounds]; prints min and median per config."""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import _lab  # noqa: E402
from parallel_c_programs_amd import ops  # noqa: E402


def t_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


n = int(sys.argv[1])
labs = [int(v) for v in sys.argv[2].split(",") if v]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 8
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
c = torch.empty(n, n, device="cuda")
cfgs = {"prod": lambda: ops.sgemm_out(a, b, c)}
for v in labs:
    cfgs[f"lab{v}"] = (lambda v=v: _lab.sgemm(a, b, v, c))
cfgs["torch"] = lambda: torch.matmul(a, b, out=c)
res = {}
for _ in range(rounds):
    for k, fn in cfgs.items():
        res.setdefault(k, []).append(t_ms(fn))
for k, v in res.items():
    print(json.dumps({"cfg": k, "n": n, "ms_min": round(min(v), 4), "tflops_max": round(2.0 * n ** 3 / min(v) / 1e9, 2),
                      "tflops_median": round(2.0 * n ** 3 / statistics.median(v) / 1e9, 2)}))
