"""Banded SpMV at the reference's configuration (`./spmv 100000 401 200 100 200 10`, 61,955,590 nnz): GPU variant 0
(one wave per row, global x) vs 1 (row blocks, LDS-staged x windows), HIP-event median of 20 calls, bytes =
the compulsory value stream + x + y. Also a cold-cache pass (a 1 GiB read between calls) since the 248 MB
value stream fits the 256 MiB Infinity Cache when called back to back."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd.utils.timing import device_time_ms  # noqa: E402

dims = tuple(int(v) for v in (sys.argv[1:7] if len(sys.argv) >= 7 else (100000, 401, 200, 100, 200, 10)))
m = ops.banded_csr(*dims)
x = ops.create_vector(dims[0])
y_ref = ops.spmv(m, x)
vals, ro, xg = m.val.cuda(), m.row_ptr.cuda(), x.cuda()
scrub = torch.rand(256 << 20, device="cuda")  # 1 GiB, READ between cold calls (no dirty lines)
bytes_ = m.nnz * 4 + dims[0] * 8
for v in [int(a) for a in sys.argv[7].split(",")] if len(sys.argv) > 7 else (1, 8):  # variants, e.g. "1,8" (-1: stream floor)
    # variant -1: the streaming floor, our reduce over the same 248 MB of values (a pure read stream, no x, no y)
    fn = ((lambda: ops.reduce(vals, "sum")) if v < 0 else  # noqa: E731
          (lambda: ops.spmv_banded(vals, ro, *dims, xg, variant=v)))
    y = fn().cpu() if v >= 0 else y_ref
    ms = device_time_ms(fn, reps=20)
    cold, cold_idle = [], []
    for _ in range(5):
        # queued: the call is enqueued while the scrub still runs (s fires as the scrub ends, the kernel follows at
        # once); idle: the GPU is idle when s is recorded, so the host's launch latency is counted too
        for queued, lst in ((True, cold), (False, cold_idle)):
            torch.cuda.synchronize()
            scrub.sum()
            if not queued:
                torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            lst.append(s.elapsed_time(e))
    cold.sort()
    cold_idle.sort()
    print(json.dumps({"variant": v, "nnz": m.nnz, "warm_ms": round(ms, 4), "warm_gbps": round(bytes_ / ms / 1e6, 1),
                      "cold_ms": round(cold[2], 4), "cold_gbps": round(bytes_ / cold[2] / 1e6, 1),
                      "cold_idle_gpu_ms": round(cold_idle[2], 4),
                      "gflops_warm": round(2 * m.nnz / ms / 1e6, 1),
                      "max_abs_err_vs_host": (y - y_ref).abs().max().item()}), flush=True)
