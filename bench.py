#!/usr/bin/env python3
"""Headline benchmark: "TFLOPS SGEMM 8192^2 + GB/s reduce 1e9 f32, at 1/2/4/8 MI355X" (BASELINE.json).

One process per GPU (torchrun / torch.distributed.run, RCCL over xGMI for N>1), weak scaling: every rank
owns its own 8192x8192 fp32 operands and its own 1e9-element f32 array (4 GB, HBM-resident, generated on
device). A timed SGEMM step is one C = A @ B on the gfx950 MFMA kernel (exact fp32); a timed reduce step
is the local HBM-bound reduction kernel followed by an RCCL all-reduce of the partial, so every rank ends
the step holding the global sum of N x 1e9 values.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; W untimed warm-up steps, then EXACTLY K
timed steps bracketed by barrier + torch.cuda.synchronize() on both sides; the max over ranks is reported;
rank 0 prints ONE JSON line. `value` = whole-job SGEMM TFLOPS (sum over GPUs); the reduce/scan numbers are
extra fields of the same line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "TFLOPS SGEMM 8192^2 + GB/s reduce 1e9 f32, at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=8192, help="SGEMM M=N=K")
    ap.add_argument("--reduce-n", type=float, default=1e9, help="f32 elements reduced per GPU per step")
    ap.add_argument("--no-scan", action="store_true", help="skip the extra prefix-scan measurement")
    ap.add_argument("--no-ref", action="store_true", help="skip the torch.matmul (hipBLASLt) reference timing")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        dist.init_process_group("nccl", device_id=dev)

    from parallel_c_programs_amd import ops
    from parallel_c_programs_amd._native import ops as native_ops

    native_ops()  # the HIP extension must load: no silent fallback on a GPU box

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed(step_fn, steps, warmup):
        for _ in range(warmup):
            step_fn()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step_fn()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if dist is not None:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return dt.item()

    n = args.size
    a = torch.empty(n, n, device=dev)
    b = torch.empty(n, n, device=dev)
    ops.rand_uniform_(a, 1000 + rank, -1.0, 1.0)
    ops.rand_uniform_(b, 2000 + rank, -1.0, 1.0)
    c = torch.empty(n, n, device=dev)

    def gemm_step():
        ops.sgemm_out(a, b, c)

    t_gemm = timed(gemm_step, args.steps, args.warmup)
    flop = 2.0 * n * n * n
    ms_gemm = 1e3 * t_gemm / args.steps
    tflops_total = world * flop * args.steps / t_gemm / 1e12

    # correctness spot check of the timed kernel (a few rows against fp64)
    rows = torch.arange(0, n, max(1, n // 8), device=dev)
    ref = a[rows].double() @ b.double()
    rel_err = ((c[rows].double() - ref).abs().max() / ref.abs().max()).item()

    ref_tflops = None
    if not args.no_ref:
        t_ref = timed(lambda: torch.matmul(a, b, out=c), max(3, args.steps // 2), 1)
        ref_tflops = world * flop * max(3, args.steps // 2) / t_ref / 1e12
    del a, b, c, ref
    torch.cuda.empty_cache()

    # ---- global reduction: local HBM reduce + RCCL all-reduce of the partial (every rank gets the sum)
    rn = int(args.reduce_n)
    x = torch.empty(rn, device=dev)
    ops.rand_uniform_(x, 3000 + rank, 0.0, 1.0)
    total = torch.zeros((), device=dev)

    def reduce_step():
        s = ops.reduce(x, "sum")
        if dist is not None:
            dist.all_reduce(s)
        total.copy_(s)

    t_red = timed(reduce_step, args.steps, args.warmup)
    red_gbps = world * 4.0 * rn * args.steps / t_red / 1e9
    expect = 0.5 * rn * world
    red_rel = abs(total.item() - expect) / expect  # uniform[0,1) mean 0.5 (statistical check)

    scan_gbps = None
    if not args.no_scan:
        y = torch.empty_like(x)
        before = torch.zeros(1, device=dev)

        def scan_step():
            # global prefix sum over the rank-ordered concatenation: N > 1 reduce-then-scan (local HBM reduce,
            # RCCL all-gather of the N totals, single-pass scan seeded with the lower ranks' sum)
            if dist is None:
                native_ops().scan_out(x, y, False, None)
                return
            tot = ops.reduce(x, "sum").reshape(1)
            tots = torch.empty(world, device=dev)
            dist.all_gather_into_tensor(tots, tot)
            before.copy_(tots[:rank].sum().reshape(1))
            native_ops().scan_out(x, y, False, before)

        t_scan = timed(scan_step, max(2, args.steps // 2), 1)
        scan_gbps = world * 8.0 * rn * max(2, args.steps // 2) / t_scan / 1e9
        del y

    # vector all-reduce bandwidth over RCCL/xGMI (N > 1): 256 MiB of f32 per rank, ring bus bandwidth
    ar_busbw = None
    if dist is not None:
        del x
        torch.cuda.empty_cache()
        v = torch.ones(64 << 20, device=dev)
        ar_steps = max(3, args.steps // 2)
        t_ar = timed(lambda: dist.all_reduce(v), ar_steps, 1)
        ar_busbw = v.numel() * 4 * 2 * (world - 1) / world * ar_steps / t_ar / 1e9
        del v

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(tflops_total, 3),
            "unit": "TFLOPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_gemm, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (uniform[-1,1) fp32 operands generated on device)",
            "config": {
                "model": f"SGEMM {n}x{n}x{n} fp32 (v_mfma_f32_32x32x2_f32) + global reduce {rn:.0e} f32/GPU",
                "global_batch": world,
                "seq_len": None,
                "parallelism": f"dp{world}",
            },
            "sgemm_tflops_per_gpu": round(tflops_total / world, 3),
            "sgemm_max_rel_err_vs_fp64": rel_err,
            "hipblaslt_torch_matmul_tflops": None if ref_tflops is None else round(ref_tflops, 3),
            "reduce_gbps": round(red_gbps, 1),
            "reduce_ms_per_step": round(1e3 * t_red / args.steps, 4),
            "reduce_elements_per_gpu": rn,
            "reduce_rel_dev_from_expectation": red_rel,
            "scan_gbps": None if scan_gbps is None else round(scan_gbps, 1),
            "allreduce_256MiB_busbw_gbps": None if ar_busbw is None else round(ar_busbw, 1),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
