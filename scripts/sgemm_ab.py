"""Interleaved A/B of SGEMM variants at one size (random operands)."""
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

n = int(sys.argv[1]); variants = [int(v) for v in sys.argv[2].split(",")]
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
ref = (a.double() @ b.double())
flop = 2.0 * n ** 3
res = {}
for v in variants:
    c = _lab.sgemm(a, b, v)
    err = ((c.double() - ref).abs().max() / ref.abs().max()).item()
    print(json.dumps({"variant": v, "n": n, "max_rel_err": err}))
for rnd in range(4):
    for v in variants:
        res.setdefault(f"v{v}", []).append(t_ms(lambda: _lab.sgemm(a, b, v)))
    res.setdefault("torch", []).append(t_ms(lambda: a @ b))
for k, v in res.items():
    print(json.dumps({"cfg": k, "n": n, "ms": min(v), "tflops": flop / min(v) / 1e9}))
