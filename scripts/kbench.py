"""Kernel micro-benchmarks on one MI355X (interleaved A/B runs in one process, random data).

python scripts/kbench.py [--what sgemm,reduce,scan,vec] [--n 1e9] [--size 8192] [--reps 10]
Prints one JSON line per measurement.
"""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402


def timeit(fn, reps, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def emit(**kw):
    print(json.dumps(kw), flush=True)


def bench_sgemm(size, reps):
    dev = torch.device("cuda")
    for n in size:
        a = torch.rand(n, n, device=dev) * 2 - 1
        b = torch.rand(n, n, device=dev) * 2 - 1
        flop = 2.0 * n * n * n
        cands = {
            "pcmx_mfma_rs8_256": lambda: ops.sgemm(a, b, variant=16),
            "pcmx_mfma_256": lambda: ops.sgemm(a, b, variant=0),
            "pcmx_mfma_128": lambda: ops.sgemm(a, b, variant=1),
            "torch_matmul": lambda: a @ b,
        }
        if n <= 4096:
            cands["pcmx_simt"] = lambda: ops.sgemm_simt(a, b)
        for name, fn in cands.items():
            if n % 256 and "256" in name:
                continue
            med, best = timeit(fn, reps)
            emit(kernel="sgemm", impl=name, n=n, ms=med, ms_best=best, tflops=flop / med / 1e9)


def bench_stream(n, reps, what):
    dev = torch.device("cuda")
    x = torch.empty(n, device=dev)
    ops.rand_uniform_(x, 1, -1, 1)
    if "reduce" in what:
        med, best = timeit(lambda: ops.reduce(x, "sum"), reps)
        emit(kernel="reduce_sum", impl="pcmx", n=n, ms=med, ms_best=best, gbps=4 * n / med / 1e6)
        med, best = timeit(lambda: x.sum(), reps)
        emit(kernel="reduce_sum", impl="torch", n=n, ms=med, ms_best=best, gbps=4 * n / med / 1e6)
    if "scan" in what:
        y = torch.empty_like(x)
        med, best = timeit(lambda: ops.native_scan_out(x, y) if hasattr(ops, "native_scan_out") else ops.scan(x), reps)
        emit(kernel="scan", impl="pcmx", n=n, ms=med, ms_best=best, gbps=8 * n / med / 1e6)
        if n <= 500_000_000:
            med, best = timeit(lambda: torch.cumsum(x, 0), reps)
            emit(kernel="scan", impl="torch", n=n, ms=med, ms_best=best, gbps=8 * n / med / 1e6)
    if "vec" in what:
        # the production streaming ops (ticket-ordered tiles, vector.hip) against torch, interleaved over 3 rounds
        w, z = torch.empty_like(x), torch.empty_like(x)
        ops.rand_uniform_(w, 2, -1, 1)
        cases = [("vadd", 12, lambda: ops.vadd(x, w), lambda: torch.add(x, w, out=z)),
                 ("vmul", 12, lambda: ops.vmul(x, w), lambda: torch.mul(x, w, out=z)),
                 ("axpy", 12, lambda: ops.axpy_(z, 0.5, x), lambda: z.add_(x, alpha=0.5)),
                 ("copy", 8, lambda: ops.copy_(z, x), lambda: z.copy_(x)),
                 ("fill", 4, lambda: ops.fill_(z, 1.5), lambda: z.fill_(1.5))]
        for rnd in range(3):
            for name, bpe, mine, ref in cases:
                for impl, fn in (("pcmx", mine), ("torch", ref)):
                    med, best = timeit(fn, reps)
                    emit(kernel=name, impl=impl, round=rnd, n=n, ms=med, ms_best=best, gbps=bpe * n / med / 1e6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="sgemm,reduce,scan,vec")
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--size", default="8192")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    what = a.what.split(",")
    t0 = time.time()
    if "sgemm" in what:
        bench_sgemm([int(s) for s in a.size.split(",")], a.reps)
    if any(w in what for w in ("reduce", "scan", "vec")):
        bench_stream(int(a.n), a.reps, what)
    emit(done=True, wall_s=time.time() - t0)


if __name__ == "__main__":
    main()
