"""SGEMM lab: cost of the per-stage barrier of the register-staged kernel (lab variants 19 = PADA 8 waves,
11 = PADA 4 waves): full kernel vs the same kernel without its stage barrier (k0_diag bit 2; wrong result,
timing only), interleaved rounds at 8192^3."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
import _lab  # noqa: E402


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


n = 8192
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
c = torch.empty(n, n, device="cuda")
res = {}
for rnd in range(4):
    for v in (19, 11):
        for name, diag in (("full", 1), ("nobarrier", 5)):
            _lab.set_tuning((1 << 8) | 8, diag)
            res.setdefault(f"v{v}_{name}", []).append(t_ms(lambda: _lab.sgemm(a, b, v, c)))
    res.setdefault("torch", []).append(t_ms(lambda: torch.matmul(a, b, out=c)))
_lab.set_tuning((1 << 8) | 8, 1)
for k, v in res.items():
    print(json.dumps({"cfg": k, "ms": min(v), "tflops": 2.0 * n ** 3 / min(v) / 1e9}))
