"""SGEMM tile-order / memory-ceiling sweep (interleaved rounds in one process, random operands)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402,F401
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    a = torch.rand(n, n, device="cuda") * 2 - 1
    b = torch.rand(n, n, device="cuda") * 2 - 1
    flop = 2.0 * n ** 3
    configs = [(1, 8, 1), (0, 0, 1), (1, 0, 1), (0, 8, 1), (1, 4, 1), (1, 16, 1), (1, 32, 1), (0, 16, 1), (1, 8, 0)]
    res = {}
    for rnd in range(3):
        for remap, grp, kd in configs:
            _lab.set_tuning((remap << 8) | grp, kd)
            for v in (5, 4):
                key = f"v{v}_remap{remap}_g{grp}_k{kd}"
                res.setdefault(key, []).append(t_ms(lambda: _lab.sgemm(a, b, v)))
        res.setdefault("torch", []).append(t_ms(lambda: a @ b))
    _lab.set_tuning((1 << 8) | 8, 1)
    for k, v in res.items():
        print(json.dumps({"cfg": k, "ms": min(v), "tflops": flop / min(v) / 1e9}))


if __name__ == "__main__":
    main()
