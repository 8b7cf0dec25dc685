"""SGEMM ceiling diagnostics: full kernel vs MFMA-only vs MFMA+LDS (variant 5), interleaved rounds."""
import ctypes, json, sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd._native import hip_lib  # noqa: E402

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
lib = hip_lib(); lib.pcmx_sgemm_set_tuning.argtypes = [ctypes.c_int, ctypes.c_int]
a = torch.rand(n, n, device="cuda") * 2 - 1
b = torch.rand(n, n, device="cuda") * 2 - 1
if zero:
    a.zero_(); b.zero_()
flop = 2.0 * n ** 3
res = {}
for rnd in range(3):
    for name, diag in [("full", 1), ("l2res", 0), ("mfma_only", 3), ("mfma_lds", 5)]:
        lib.pcmx_sgemm_set_tuning((1 << 8) | 8, diag)
        res.setdefault(name, []).append(t_ms(lambda: ops.sgemm(a, b, variant=5)))
    res.setdefault("torch", []).append(t_ms(lambda: a @ b))
lib.pcmx_sgemm_set_tuning((1 << 8) | 8, 1)
for k, v in res.items():
    print(json.dumps({"cfg": k, "zero": zero, "ms": min(v), "tflops": flop / min(v) / 1e9}))
