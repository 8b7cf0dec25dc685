#!/usr/bin/env python3
"""Headline benchmark: "TFLOPS SGEMM 8192^2 + GB/s reduce 1e9 f32, at 1/2/4/8 MI355X" (BASELINE.json), plus
every other BASELINE.json north-star config measured at the same N in the same job.

One process per GPU (torchrun / torch.distributed.run, RCCL over xGMI for N > 1). Sections, each with its
own correctness check, all timed the same way (W untimed warm-up steps, then EXACTLY K timed steps bracketed
by barrier + torch.cuda.synchronize() on both sides, max over ranks; utils/harness.py):

  sgemm    (value) 8192^3 fp32 C = A @ B per GPU on the MFMA kernel, weak scaling; fp64 spot check; the
           hipBLASLt torch.matmul of the same operands is timed alongside for reference, and so is the fp32 GEMM on
           the bf16 matrix cores (exact 3-way operand split, 6 piece products: fp32 accuracy, its own fp64 check;
           an extra field, never the headline value)
  reduce   global sum, local HBM reduce + one-scalar RCCL all-reduce: weak (1e9 f32 per GPU) and strong
           (1e9 f32 in total, 1e9/N per GPU); fp64 check
  scan     global inclusive prefix sum over the rank-ordered concatenation (reduce-then-scan): weak and
           strong like reduce; fp64 check of EVERY output of every rank incl. its rank offset, after the stream's
           look-back error word (scan_check)
  stencil  16384^2 bf16 5-point stencil, strong scaling: row slabs, T fused updates per kernel (T by slab
           height: 8 / 8 / 6 / 6 at N = 1 / 2 / 4 / 8) and one T-row halo exchange per neighbour overlapped with
           the interior update; bit-exact checks: the timed grid itself (all warm-up + timed updates) against a
           plain-PyTorch single-step oracle, and a small grid through the same distributed path
  spmv     power-law CSR, 1e8 nnz / 1e7 rows, strong scaling: nnz-balanced row blocks, XCD-sliced kernel,
           ghost exchange (only the x entries each rank's nonzeros reference, grouped per-peer send/recv) chunked
           and overlapped with the product; fp64 check of every rank's rows
  (N > 1)  256 MiB RCCL all-reduce bus bandwidth
  vendor   every section carries the vendor library on the same data, timed identically: hipBLASLt
           (torch.matmul), rocPRIM (torch.sum, torch.cumsum), hipSPARSE (torch sparse CSR x vector) and, at N = 1,
           rocSPARSE's generic SpMV with its analysis done once (bin/spmv_vendor, a child process)

rank 0 prints ONE JSON line; `value` = whole-job SGEMM TFLOPS (sum over GPUs), the other configs are extra
fields of the same line. A section after SGEMM that raises is reported as "<section>_error" in the line (its
fields missing) instead of costing the line. `--small` shrinks every size (CPU/gloo rehearsal of the multi-rank path, tests).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "TFLOPS SGEMM 8192^2 + GB/s reduce 1e9 f32, at 1/2/4/8 MI355X"
SECTIONS = ("sgemm", "reduce", "scan", "stencil", "spmv")


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=8192, help="SGEMM M=N=K")
    ap.add_argument("--reduce-n", type=float, default=1e9, help="f32 elements (per GPU weak, in total strong)")
    ap.add_argument("--stencil-n", type=int, default=16384)
    ap.add_argument("--stencil-fuse", type=int, default=0,
                    help="fused updates per kernel / halo depth (0: by slab height, 8 / 8 / 6 / 6 at N = 1 / 2 / 4 / 8)")
    ap.add_argument("--spmv-rows", type=float, default=1e7)
    ap.add_argument("--spmv-nnz", type=float, default=1e8)
    ap.add_argument("--spmv-chunks", type=int, default=0, help="exchange pipeline depth (0: 1 at N=1, else 2)")
    ap.add_argument("--spmv-exchange", default="ghost", choices=("ghost", "allgather"),
                    help="N>1 vector exchange: only the referenced entries (ghost) or the whole y (allgather)")
    ap.add_argument("--sections", default=",".join(SECTIONS), help="comma list out of " + ",".join(SECTIONS))
    ap.add_argument("--no-ref", action="store_true", help="skip the torch.matmul (hipBLASLt) reference timing")
    ap.add_argument("--no-x6", action="store_true", help="skip the fp32-via-bf16x6 SGEMM extra (variant 20)")
    ap.add_argument("--small", action="store_true", help="tiny sizes (CPU/gloo rehearsal)")
    ap.add_argument("--device", default=None, help="cuda (default when a GPU is visible) or cpu")
    ap.add_argument("--backend", default=None, choices=("nccl", "gloo"),
                    help="process-group backend (default: nccl = RCCL on a GPU). gloo with --device cuda runs every "
                         "rank's GPU kernels with host-staged messages: N ranks on ONE GPU (tests of the N>1 path)")
    a = ap.parse_args(argv)
    if a.small:
        a.size, a.reduce_n, a.stencil_n, a.spmv_rows, a.spmv_nnz = 256, 1e5, 256, 2e4, 2e5
    return a


def _r(v, nd=4):
    """Round to nd decimals, keeping at least 4 significant digits (tiny CPU-rehearsal values stay nonzero)."""
    if v is None:
        return None
    v = float(v)
    return round(v, nd) if abs(v) >= 10 ** (3 - nd) else float(f"{v:.4g}")


def rocsparse_bar(n_rows: int, nnz: int, reps: int) -> dict:
    """rocSPARSE's generic SpMV (preprocess once, compute stage timed) on the same power-law matrix: bin/spmv_vendor,
    a child process on /opt/rocm's rocSPARSE + HIP runtime (torch's sparse CSR path re-analyses the matrix per call).
    Runs after our sections, this process idle on the GPU meanwhile."""
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bin", "spmv_vendor")
    if not os.path.exists(exe):
        return {"rocsparse_spmv_gflops": "not built (bin/spmv_vendor)"}
    try:
        r = subprocess.run([exe, str(n_rows), str(nnz), str(reps)], capture_output=True, text=True, timeout=240)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        res = json.loads(line)
        algs = {k[:-7]: v for k, v in res.items() if k.endswith("_gflops") and k != "best_gflops"}
        best = max(algs, key=algs.get)
        return {"rocsparse_spmv_gflops": res["best_gflops"], "rocsparse_spmv_alg": best,
                "rocsparse_spmv_max_rel_err": res.get(f"{best}_max_rel_err")}
    except Exception as e:  # the line says why the bar is missing
        return {"rocsparse_spmv_gflops": f"failed: {type(e).__name__}: {e}"[:200]}


def main(argv=None):
    args = parse(argv)
    from parallel_c_programs_amd.models import workloads as W
    from parallel_c_programs_amd.parallel import finalize, init
    from parallel_c_programs_amd.utils.harness import timed
    from parallel_c_programs_amd.utils.metrics import bench_line

    ctx = init(backend=args.backend, device=args.device)
    world, rank, dev = ctx.world, ctx.rank, ctx.device
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if dev.type == "cuda":
        from parallel_c_programs_amd._native import ops as native_ops

        native_ops()  # the HIP extension must load: no silent fallback on a GPU box
    sections = [s for s in args.sections.split(",") if s]
    K, Wm = args.steps, args.warmup
    out = {}

    def free():
        if dev.type == "cuda":
            torch.cuda.empty_cache()

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    # ---- SGEMM (headline value): weak scaling, 8192^3 per GPU
    n = args.size
    tflops = ms_gemm = None
    if "sgemm" in sections:
        g = W.Sgemm(ctx, n=n)
        t = timed(ctx, g.step, K, Wm)
        rep = g.report(t, K)
        tflops, ms_gemm = rep["value"], rep["ms_per_step"]
        out["sgemm_tflops_per_gpu"] = _r(tflops / world, 3)
        out["sgemm_max_rel_err_vs_fp64"] = ctx.max_over_ranks(g.check()["max_rel_err_vs_fp64"])
        if not args.no_ref and dev.type == "cuda":
            # the vendor library timed exactly like our kernel (same warm-up and step count)
            t_ref = timed(ctx, lambda: torch.matmul(g.a, g.b, out=g.c), K, Wm)
            out["hipblaslt_torch_matmul_tflops"] = _r(world * g.work_per_step() * K / t_ref / 1e12, 3)
        if not args.no_x6 and dev.type == "cuda" and n % 256 == 0:
            # fp32 GEMM on the bf16 matrix cores (exact 3-way operand split, 6 piece products; sgemm_x6.hip): an
            # fp32-accurate extra, timed identically with its own fp64 check; never the headline value. A failure
            # here costs only these fields (the headline above is already measured)
            try:
                g.variant = 20
                t_x6 = timed(ctx, g.step, K, Wm)
                out["sgemm_fp32_via_bf16x6_tflops"] = _r(world * g.work_per_step() * K / t_x6 / 1e12, 3)
                out["sgemm_fp32_via_bf16x6_max_rel_err_vs_fp64"] = ctx.max_over_ranks(
                    g.check()["max_rel_err_vs_fp64"])
            except Exception as e:  # noqa: BLE001 - reported in the JSON line
                out["sgemm_fp32_via_bf16x6_error"] = f"{type(e).__name__}: {e}"[:300]
        del g
        free()
        log(f"sgemm {tflops:.1f} TFLOPS")

    def guarded(name, fn):
        """Runs one extra section; an exception (raised on every rank alike, e.g. a shape or check failure) is
        recorded as "<name>_error" in the line instead of costing the whole line (the headline SGEMM value and the
        other sections still report). A section that hangs is not caught: the driver's time limit ends the run."""
        try:
            fn()
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            out[f"{name}_error"] = f"{type(e).__name__}: {e}"[:300]
            log(f"{name} FAILED: {out[name + '_error']}")
        free()  # (after the except block: the traceback no longer pins the section's tensors)

    # ---- reduce / scan: weak (rn per GPU) and strong (rn in total); identical runs at N = 1
    rn = int(args.reduce_n)

    def reduce_scan(name, cls):
        for mode, per_rank in (("weak", rn), ("strong", -(-rn // world))):
            if mode == "strong" and world == 1:
                for k in ("gbps", "ms_per_step", "rel_err_vs_fp64"):
                    out[f"{name}_strong_{k}"] = out[f"{name}_weak_{k}"]
                continue
            w = cls(ctx, n=per_rank)
            t = timed(ctx, w.step, K, Wm)
            rep = w.report(t, K)
            out[f"{name}_{mode}_gbps"] = _r(rep["value"], 1)
            out[f"{name}_{mode}_ms_per_step"] = _r(rep["ms_per_step"])
            out[f"{name}_{mode}_rel_err_vs_fp64"] = ctx.max_over_ranks(w.check()["rel_err_vs_fp64"])
            if mode == "weak" and not args.no_ref and dev.type == "cuda":
                # the vendor library on the same per-GPU data, timed exactly like our kernel (rocPRIM behind both)
                if name == "reduce":
                    t_ref = timed(ctx, lambda: torch.sum(w.x), K, Wm)
                    out["torch_sum_gbps"] = _r(world * 4.0 * w.x.numel() * K / t_ref / 1e9, 1)
                else:
                    ybuf = torch.empty_like(w.x)
                    t_ref = timed(ctx, lambda: torch.cumsum(w.x, 0, out=ybuf), K, Wm)
                    out["torch_cumsum_gbps"] = _r(world * 8.0 * w.x.numel() * K / t_ref / 1e9, 1)
                    del ybuf
            if name == "scan":  # every timed output checked (not a prefix), rank offsets included
                out["scan_full_max_rel_err_vs_fp64"] = max(out.get("scan_full_max_rel_err_vs_fp64", 0.0),
                                                           out[f"scan_{mode}_rel_err_vs_fp64"])
            del w
            free()
        log(f"{name} weak {out[name + '_weak_gbps']} GB/s, strong {out[name + '_strong_gbps']} GB/s")

    for name, cls in (("reduce", W.Reduce), ("scan", W.Scan)):
        if name in sections:
            guarded(name, lambda: reduce_scan(name, cls))

    # ---- stencil 16384^2 bf16, strong scaling over row slabs with the overlapped fused halo exchange
    def stencil():
        s = W.Stencil(ctx, n=args.stencil_n, fuse=args.stencil_fuse)
        t = timed(ctx, s.step, K, Wm)
        rep = s.report(t, K)
        chk = s.check()
        out.update({"stencil_glups": _r(rep["value"], 1), "stencil_ms_per_step": _r(rep["ms_per_step"]),
                    "stencil_updates_per_step": s.slab.fuse,
                    "stencil_timed_grid_bit_exact": chk["timed_grid_bit_exact"],
                    "stencil_timed_grid_updates": chk["timed_grid_updates"],
                    "stencil_bit_exact": chk["bit_exact_vs_single_step_oracle"], "stencil_finite": chk["finite"]})
        del s
        log(f"stencil {out['stencil_glups']} GLUP/s")

    if "stencil" in sections:
        guarded("stencil", stencil)

    # ---- SpMV 1e8-nnz power-law graph, strong scaling
    def spmv():
        vendor = not args.no_ref and dev.type == "cuda"
        sp = W.SpMV(ctx, n_rows=int(args.spmv_rows), nnz=int(args.spmv_nnz), chunks=args.spmv_chunks,
                    exchange=args.spmv_exchange, keep_plain=vendor)
        t = timed(ctx, sp.step, K, Wm)
        rep = sp.report(t, K)
        out.update({"spmv_gflops": _r(rep["value"], 2), "spmv_ms_per_step": _r(rep["ms_per_step"]),
                    "spmv_effective_gbps": _r(rep["effective_gbps"], 1), "spmv_chunks": sp.d.chunks, "spmv_slices": sp.d.slices,
                    "spmv_exchange": sp.d.exchange if ctx.distributed else None,
                    "spmv_max_rel_err_vs_fp64": sp.check()["max_rel_err_vs_fp64"]})
        if vendor:  # hipSPARSE (torch sparse CSR x dense vector) on each rank's own rows, the same matrix and x
            try:
                A = sp.d.vendor_matrix()
                yv = torch.mv(A, sp.xp)
                t_ref = timed(ctx, lambda: torch.mv(A, sp.xp), K, Wm)
                nnz_all = ctx.scalar(float(sp.d.local_nnz))
                ctx.all_reduce_(nnz_all)
                out["torch_sparse_csr_gflops"] = _r(2.0 * nnz_all.item() * K / t_ref / 1e9, 2)
                del A, yv
            except Exception as e:  # the line says so instead of dropping the bar
                out["torch_sparse_csr_gflops"] = f"unsupported on this torch build: {type(e).__name__}: {e}"[:200]
        del sp
        free()
        log(f"spmv {out['spmv_gflops']} GFLOP/s")
        if vendor and world == 1:
            out.update(rocsparse_bar(int(args.spmv_rows), int(args.spmv_nnz), K))

    if "spmv" in sections:
        guarded("spmv", spmv)

    # ---- RCCL all-reduce bus bandwidth over xGMI (N > 1)
    def allreduce():
        import torch.distributed as dist

        v = torch.ones(64 << 20, device=dev)
        kr = max(3, K // 2)
        t_ar = timed(ctx, lambda: dist.all_reduce(v), kr, 1)
        out["allreduce_256MiB_busbw_gbps"] = _r(v.numel() * 4 * 2 * (world - 1) / world * kr / t_ar / 1e9, 1)

    if ctx.distributed and dev.type == "cuda" and ctx.backend == "nccl":
        guarded("allreduce", allreduce)

    rc = 0
    if rank == 0:
        # BASELINE.json publishes no number ("published": {}), so vs_baseline stays null
        fields = dict(
            metric=METRIC, value=_r(tflops, 3), unit="TFLOPS", n_gpus=world, steps=K, warmup=Wm,
            ms_per_step=_r(ms_gemm), higher_is_better=True, scaling="weak", baseline=None, dtype="fp32",
            data="synthetic (uniform random operands generated on device; power-law CSR generated per rank)",
            config={
                "model": f"SGEMM {n}x{n}x{n} fp32 (v_mfma_f32_32x32x2_f32) per GPU + global reduce/scan "
                         f"{rn:.0e} f32 + stencil {args.stencil_n}^2 bf16 + SpMV {args.spmv_nnz:.0e} nnz",
                "global_batch": world,
                "seq_len": None,
                "parallelism": f"dp{world}",
            },
            device=dev.type, **out)
        try:
            line = bench_line(partial="sgemm" not in sections, **fields)
        except ValueError as e:  # still print what was measured (with the reason), then fail the run after finalize
            line = {k: v for k, v in fields.items() if k != "baseline"}
            line["vs_baseline"] = None
            line["contract_error"], rc = str(e), 1
        print(json.dumps(line), flush=True)
    finalize(ctx)  # every rank reaches this, also when rank 0's line failed the contract
    return rc


if __name__ == "__main__":
    sys.exit(main())
