"""SGEMM ceiling diagnostics: full kernel vs MFMA-only vs MFMA+LDS (variant 5), interleaved rounds."""
import json, sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402,F401
sys.path.insert(0, str(Path(__file__).resolve().parent))
import _lab  # noqa: E402

def t_ms(fn, reps=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / reps

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
zero = len(sys.argv) > 2 and sys.argv[2] == "zero"
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
if zero:
    a.zero_(); b.zero_()
flop = 2.0 * n ** 3
res = {}
for rnd in range(3):
    for name, diag in [("full", 1), ("l2res", 0), ("mfma_only", 3), ("mfma_lds", 5)]:
        _lab.set_tuning((1 << 8) | 8, diag)
        res.setdefault(name, []).append(t_ms(lambda: _lab.sgemm(a, b, 5)))
    res.setdefault("torch", []).append(t_ms(lambda: a @ b))
_lab.set_tuning((1 << 8) | 8, 1)
for k, v in res.items():
    print(json.dumps({"cfg": k, "zero": zero, "ms": min(v), "tflops": flop / min(v) / 1e9}))
