#!/usr/bin/env python3
"""Headline benchmark: "TFLOPS SGEMM 8192^2 + GB/s reduce 1e9 f32, at 1/2/4/8 MI355X" (BASELINE.json), plus
every other BASELINE.json north-star config measured at the same N in the same job.

One process per GPU over RCCL/xGMI. `bench.py --gpus N` with N > 1 and no launcher environment (no WORLD_SIZE)
starts `python -m torch.distributed.run --nproc-per-node N bench.py ...` itself as a child process, before anything
touches the GPU, and exits with its status (the reference's `mpirun -n P region pic1.bmp`,
2-mpi-region-growing/Makefile:4); N larger than the visible GPU count is refused, and so is a launcher whose
WORLD_SIZE differs from --gpus. Sections, each with its own correctness check, all timed the same way (W untimed
warm-up steps, then EXACTLY K timed steps bracketed by barrier + torch.cuda.synchronize() on both sides, max over
ranks; utils/harness.py; on a GPU each section's W warm-ups follow --settle-ms (30) of untimed steps, so the timed
steps run at the steady-state shader clock), each also reporting its per-step hipEvent device time (min / median /
max) and its longest host enqueue:

  sgemm    (value) 8192^3 fp32 C = A @ B per GPU on the MFMA kernel, weak scaling; EVERY element of C checked
           against an fp64 GEMM; the hipBLASLt torch.matmul of the same operands is timed alongside for reference,
           and so is the fp32 GEMM on the bf16 matrix cores (exact 3-way operand split, 6 piece products: fp32
           accuracy, its own full fp64 check; an extra field, never the headline value)
  reduce   global sum, local HBM reduce + one-scalar RCCL all-reduce (left in flight behind the next step's local
           reduce, completed inside the timed region): weak (1e9 f32 per GPU) and strong (1e9 f32 in total, 1e9/N
           per GPU); fp64 check of the last step's global total
  scan     global inclusive prefix sum over the rank-ordered concatenation (reduce-then-scan): weak and
           strong like reduce; fp64 check of EVERY output of every rank incl. its rank offset, and the stream's
           look-back error word
  axpy     y <- alpha x + y, 1e9 f32 per GPU (12 B/element), weak scaling, no communication; every element of the
           timed output checked against fp64 (data chosen so that every step is exact in fp32); torch's
           y.add_(x, alpha=a) timed alongside
  stencil  16384^2 bf16 5-point stencil (random grid), strong scaling: row slabs, T fused updates per kernel (T by
           slab height: 8 / 8 / 6 / 6 at N = 1 / 2 / 4 / 8), a deep halo at N = 4 / 8 (5T rows exchanged every 5th
           step, overlapped with the interior update; self-tested on the job's backend first); bit-exact checks: the timed grid itself (all warm-up + timed updates) against a
           plain-PyTorch single-step oracle, and a small grid through the same distributed path
  spmv     power-law CSR, 1e8 nnz / 1e7 rows, strong scaling: nnz-balanced row blocks, XCD-sliced kernel,
           ghost exchange (only the x entries each rank's nonzeros reference, grouped per-peer send/recv) chunked
           and overlapped with the product; fp64 check of every rank's rows and ghosts
  (N > 1)  256 MiB RCCL all-reduce bus bandwidth
  vendor   every section carries the vendor library on the same data: hipBLASLt (torch.matmul), rocPRIM
           (torch.sum, torch.cumsum), hipSPARSE (torch sparse CSR x vector) timed like our kernels, and rocSPARSE's
           generic SpMV with its analysis done once (bin/spmv_vendor, a child process per rank: W warm-ups, then K
           back-to-back calls between two events, the mean; fp64 reference; at N > 1 each rank's local product, no
           exchange, the slowest rank's time)

Checks are ENFORCED: fp64-referenced errors must be <= 1e-5 (workloads.REL_ERR_LIMIT), bit-exact flags true. A
failing check adds "<section>_check_failed" (the failing keys) to the line; a section that raises adds
"<section>_error". Either way the line is still printed once by rank 0, every rank records the same outcome (a
collective decision on a separate CPU process group at the end of each section: a failure local to one rank cannot
pair with a data collective another rank waits in; a rank that fails before a timed region stops the others at the
next decision point, Runner), and the run exits 1. `--inject-fault SECTION:RANK:KIND` (KIND perturb = corrupt that
rank's timed output after timing, raise = raise in its check, raise-early = raise right after its set-up, before the
timed region, selftest = report the stencil / SpMV N > 1 self-test as failed) is the test hook.

At N > 1 every distributed section (reduce, scan, stencil, spmv) also times its COMPUTE-ONLY twin in the same job
(the same kernels on the same data, the exchange skipped) and reports <section>_compute_only_ms,
<section>_comm_exposed_ms, the per-rank spread of its median device step time and the bytes each rank exchanges per
step (attribute_comm), plus the process group's backend and size (comm_backend, comm_world_size): a first
multi-GPU run then says whether a miss is exposed communication, imbalance between ranks or compute.

rank 0 prints ONE JSON line; `value` = whole-job SGEMM TFLOPS (sum over GPUs), the other configs are extra fields
of the same line. `--small` shrinks every size (CPU/gloo rehearsal of the multi-rank path, tests).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "TFLOPS SGEMM 8192^2 + GB/s reduce 1e9 f32, at 1/2/4/8 MI355X"
SECTIONS = ("sgemm", "reduce", "scan", "axpy", "stencil", "spmv")


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under a launcher, else 1); N > 1 without a launcher "
                         "starts torch.distributed.run itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-ms", type=float, default=30.0,
                    help="GPU: untimed steps for this much wall time before each section's W warm-up steps, so the "
                         "timed steps run at the steady-state clock (0: off)")
    ap.add_argument("--size", type=int, default=8192, help="SGEMM M=N=K")
    ap.add_argument("--reduce-n", type=float, default=1e9, help="f32 elements (per GPU weak, in total strong)")
    ap.add_argument("--stencil-n", type=int, default=16384)
    ap.add_argument("--stencil-fuse", type=int, default=0,
                    help="fused updates per kernel / halo depth (0: by slab height, 8 / 8 / 6 / 6 at N = 1 / 2 / 4 / 8)")
    ap.add_argument("--stencil-halo-mult", type=int, default=0,
                    help="deep halo: m x fuse halo rows exchanged every m steps (0: auto, 5 on slabs of <= 4096 rows at N > 1, else 1)")
    ap.add_argument("--spmv-rows", type=float, default=1e7)
    ap.add_argument("--spmv-nnz", type=float, default=1e8)
    ap.add_argument("--spmv-chunks", type=int, default=0, help="exchange pipeline depth (0: 1 at N=1, else 2)")
    ap.add_argument("--spmv-exchange", default="ghost", choices=("ghost", "allgather"),
                    help="N>1 vector exchange: only the referenced entries (ghost) or the whole y (allgather)")
    ap.add_argument("--sections", default=",".join(SECTIONS), help="comma list out of " + ",".join(SECTIONS))
    ap.add_argument("--no-ref", action="store_true", help="skip the vendor-library timings")
    ap.add_argument("--no-x6", action="store_true", help="skip the fp32-via-bf16x6 SGEMM extra (variant 20)")
    ap.add_argument("--small", action="store_true", help="tiny sizes (CPU/gloo rehearsal)")
    ap.add_argument("--device", default=None, help="cuda (default when a GPU is visible) or cpu")
    ap.add_argument("--backend", default=None, choices=("nccl", "gloo"),
                    help="process-group backend (default: nccl = RCCL on a GPU). gloo with --device cuda runs every "
                         "rank's GPU kernels with host-staged messages: N ranks may share ONE GPU (tests of the N>1 "
                         "path)")
    ap.add_argument("--inject-fault", default=None, metavar="SECTION:RANK:KIND",
                    help="test hook: KIND perturb (corrupt that rank's timed output), raise (raise in its check) or "
                         "raise-early (raise after its set-up, before the timed region)")
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


# ------------------------------------------------------------------------------------------------ launcher
def _wants_gpu(args) -> bool:
    if args.device is not None:
        return args.device.startswith("cuda")
    return torch.cuda.device_count() > 0  # (counts devices without initialising HIP in this process)


def launch(args, argv: list[str]) -> int:
    """--gpus N > 1 without a launcher: one fresh `torch.distributed.run` child with N ranks (this process never
    touches the GPU and never execs), its exit status returned. Each rank's stdout goes straight through; only rank 0
    prints the JSON line."""
    if _wants_gpu(args) and args.backend != "gloo":
        visible = torch.cuda.device_count()
        if args.gpus > visible:
            print(f"[bench] error: --gpus {args.gpus} but only {visible} GPU(s) visible; one rank per GPU over RCCL "
                  f"needs {args.gpus} (--backend gloo lets ranks share a GPU, for tests)", file=sys.stderr, flush=True)
            return 2
    from parallel_c_programs_amd.parallel.dist import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    print(f"[bench] launching {args.gpus} ranks: torch.distributed.run --nproc-per-node {args.gpus}", file=sys.stderr,
          flush=True)
    rc = subprocess.run(cmd, env=env).returncode
    return rc if rc >= 0 else 128 - rc


def rocsparse_bar(n_rows: int, nnz: int, reps: int, warmup: int, rows: tuple[int, int] | None = None,
                  device: int | None = None) -> dict:
    """rocSPARSE's generic SpMV (preprocess once; W warm-up calls, then K back-to-back compute calls between two
    events, the mean; max error against an fp64 host product) on the same power-law matrix: bin/spmv_vendor, a
    child process on /opt/rocm's rocSPARSE + HIP runtime (torch's sparse CSR path re-analyses the matrix per call).
    Runs after our sections, this process idle on the GPU meanwhile. rows=(row0, row1), device: one rank's block
    of rows (its local product, no exchange) on that rank's GPU; the result then also holds per-algorithm ms."""
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bin", "spmv_vendor")
    if not os.path.exists(exe):
        return {"rocsparse_spmv_gflops": "not built (bin/spmv_vendor)"}
    try:
        cmd = [exe, str(n_rows), str(nnz), str(reps), str(warmup)]
        if rows is not None:
            cmd += [str(rows[0]), str(rows[1])] + ([str(device)] if device is not None else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        res = json.loads(line)
        algs = {k[:-7]: v for k, v in res.items() if k.endswith("_gflops") and k != "best_gflops"}
        best = max(algs, key=algs.get)
        return {"rocsparse_spmv_gflops": res["best_gflops"], "rocsparse_spmv_alg": best,
                "rocsparse_spmv_max_rel_err_vs_fp64": res.get(f"{best}_max_rel_err"),
                "_ms": {a: res[f"{a}_ms"] for a in algs}, "_nnz": res["nnz"]}
    except Exception as e:  # the line says why the bar is missing
        return {"rocsparse_spmv_gflops": f"failed: {type(e).__name__}: {e}"[:200]}


def ranks_share_gpu(ctx) -> bool:
    """More ranks on this node than GPUs (gloo rehearsals): the same answer on every rank of the node."""
    return ctx.distributed and int(os.environ.get("LOCAL_WORLD_SIZE", ctx.world)) > torch.cuda.device_count()


def rocsparse_bar_ranks(ctx, n_rows: int, nnz: int, reps: int, warmup: int, rows: tuple[int, int]) -> dict:
    """N > 1: every rank runs rocSPARSE on its own block of rows (bin/spmv_vendor with a row range, on its own GPU),
    all ranks at once after a barrier; per algorithm the job's time is the SLOWEST rank's (as for our step) and the
    GFLOP/s the whole matrix's 2 nnz over it. Compute only (no exchange): a bar our full step has to beat with its
    exchange included. Every rank makes the same collectives whether or not its child process succeeded. Ranks that
    share a GPU (gloo rehearsals) skip it: a child per rank would double the processes on that GPU."""
    if ranks_share_gpu(ctx):
        return {"rocsparse_spmv_gflops": "not measured: ranks share a GPU"}
    ctx.barrier()
    res = rocsparse_bar(n_rows, nnz, reps, warmup, rows=rows, device=ctx.device.index)
    names = ("csr_adaptive", "csr_rowsplit")
    ms = [float(res.get("_ms", {}).get(a, float("inf"))) for a in names]
    worst = [ctx.max_over_ranks(v) for v in ms]
    nnz_all = ctx.scalar(float(res.get("_nnz", 0)))
    ctx.all_reduce_(nnz_all)
    err = ctx.max_over_ranks(float(res.get("rocsparse_spmv_max_rel_err_vs_fp64") or 0.0))
    gf = {a: 2.0 * nnz_all.item() / (w * 1e-3) / 1e9 for a, w in zip(names, worst) if w != float("inf")}
    if not gf:  # (the same answer on every rank)
        return {"rocsparse_spmv_gflops": "failed on a rank (bin/spmv_vendor child process)"}
    best = max(gf, key=gf.get)
    return {"rocsparse_spmv_gflops": _r(gf[best], 2), "rocsparse_spmv_alg": best,
            "rocsparse_spmv_max_rel_err_vs_fp64": err, "rocsparse_spmv_scope": "local products, no exchange"}


# ------------------------------------------------------------------------------------------------ sections
class Checks:
    """One section's local check values: record(key, value, limit) with value <= limit to pass (errors), or a bool
    that must be True (bit-exact flags); info(key, value, agg) for reported-only values (device step times)."""

    def __init__(self):
        self.items = {}  # key -> (value, agg, limit)

    def error(self, key, value, limit):
        self.items[key] = (float(value), "max", float(limit))

    def flag(self, key, ok):
        self.items[key] = (bool(ok), "all", None)

    def info(self, key, value, agg="max"):
        """agg over ranks: "max", "min" or "sum"."""
        self.items[key] = (value, agg, None)


class PeerFailed(Exception):
    """Raised at a decision point when another rank's section has already failed."""


class Runner:
    """Runs bench sections. A section is a generator: every `yield` is a DECISION POINT (before each timed region and
    before the checks), where all ranks join one all_gather_object on a separate gloo group. A rank whose section
    raised no longer yields: it enters the FINAL exchange (its error and local check values), repeated until every
    rank is final. A healthy rank that meets a failed peer's final message at a decision point stops its section there
    (PeerFailed) and turns final too, so a rank that failed early is reported and the others do not walk into a data
    collective it will never join. All ranks then merge the same final states and record the same outcome. (A failure
    INSIDE a data collective sequence — one rank raising between two collectives with no decision point in between —
    still ends the job through the process group's timeout, PCMX_PG_TIMEOUT_S.)"""

    def __init__(self, ctx, out: dict, fault: str | None, log):
        from parallel_c_programs_amd.parallel.dist import side_group

        self.ctx, self.out, self.log = ctx, out, log
        self.side = side_group(ctx)
        self.failed = []  # sections that errored or failed a check
        self.fault = None
        if fault:
            sec, rank, kind = fault.split(":")
            if kind not in ("perturb", "raise", "raise-early", "selftest"):
                raise ValueError("--inject-fault SECTION:RANK:perturb|raise|raise-early|selftest")
            self.fault = (sec, int(rank), kind)

    def injected(self, section: str, kind: str) -> bool:
        return self.fault is not None and self.fault == (section, self.ctx.rank, kind)

    def maybe_raise(self, section: str, kind: str = "raise"):
        if self.injected(section, kind):
            raise RuntimeError(f"injected fault in {section} on rank {self.ctx.rank}")

    def run(self, name: str, fn) -> None:
        from parallel_c_programs_amd.parallel.dist import gather_objects

        chk, err = Checks(), None
        try:
            for _ in fn(chk):  # a decision point
                states = gather_objects(("point", None, None), self.side)
                bad = [r for r, (kind, e, _) in enumerate(states) if kind == "final"]
                if bad:
                    raise PeerFailed(f"rank {bad[0]} failed earlier in the section")
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            err = f"{type(e).__name__}: {e}"[:300]
        if self.ctx.device.type == "cuda":
            torch.cuda.empty_cache()  # (after the except block: no traceback pins the section's tensors)
        while True:  # the final exchange, until every rank has left its section
            states = gather_objects(("final", err, chk.items), self.side)
            if all(kind == "final" for kind, _, _ in states):
                break
        errs = [(r, e) for r, (_, e, _) in enumerate(states) if e and not e.startswith("PeerFailed")]
        errs = errs or [(r, e) for r, (_, e, _) in enumerate(states) if e]
        if errs:
            r, e = errs[0]
            self.out[f"{name}_error"] = e if r == 0 and len(errs) == 1 else f"rank {r}: {e}" + (
                f" (+{len(errs) - 1} more ranks)" if len(errs) > 1 else "")
        merged = {}
        for _, _, items in states:
            for k, (v, agg, limit) in items.items():
                if k not in merged:
                    merged[k] = (v, agg, limit)
                    continue
                pv = merged[k][0]
                merged[k] = ((pv and v) if agg == "all" else max(pv, v) if agg == "max" else pv + v if agg == "sum"
                             else min(pv, v), agg, limit)
        bad = []
        for k, (v, agg, limit) in merged.items():
            self.out[k] = _r(v, 4) if agg in ("max", "min", "sum") and limit is None else v
            if (agg == "all" and not v) or (limit is not None and not v <= limit):
                bad.append(k)
        if bad:
            self.out[f"{name}_check_failed"] = bad
        if errs or bad:
            self.failed.append(name)
            self.log(f"{name} FAILED: " + (self.out.get(f"{name}_error", "") + " " + " ".join(bad)).strip())


def device_times(chk: Checks, prefix: str, ms: list, hms: list | None = None) -> None:
    """Per-step device times (min / median / max over steps, max over ranks) and the longest host enqueue of a step:
    a device_ms_max outlier with a small host_ms_max is a device-side stall, not the Python host."""
    from parallel_c_programs_amd.utils.harness import step_stats

    for k, v in step_stats(ms).items():
        chk.info(f"{prefix}_device_ms_{k}", v, "max")
    if hms:
        chk.info(f"{prefix}_host_ms_max", max(hms), "max")


def attribute_comm(ctx, chk: Checks, out: dict, prefix: str, full_ms: float, dev_ms: list, w, steps: int,
                   warmup: int, settle_ms: float) -> None:
    """N > 1: what a step's time is made of, measured in the same job (so a first multi-GPU run explains itself):
      <prefix>_compute_only_ms      the same kernels on the same data with every exchange skipped (w.compute_only_step),
                                    timed exactly like the full step (W warm-ups, K steps between barrier + sync, max
                                    over ranks);
      <prefix>_comm_exposed_ms      full step minus compute-only: the communication the schedule did not hide;
      <prefix>_rank_step_ms_min/max the per-rank median device step time, lowest and highest rank (imbalance), for
                                    the full step and (…_compute_only_rank_ms_min/max) the compute-only twin;
      <prefix>_bytes_exchanged_per_step          the most one rank sends per step (payload bytes);
      <prefix>_bytes_exchanged_per_step_total    summed over ranks.
    Runs AFTER the section's checks: the twin leaves the data unchecked (stale halos / ghosts)."""
    import statistics

    from parallel_c_programs_amd.utils.harness import timed

    ms_c = []
    t = timed(ctx, w.compute_only_step, steps, warmup, ms_c, settle_ms=settle_ms)
    comp = 1e3 * t / steps
    out[f"{prefix}_compute_only_ms"] = _r(comp)
    out[f"{prefix}_comm_exposed_ms"] = _r(full_ms - comp)
    if dev_ms:
        med = statistics.median(dev_ms)
        chk.info(f"{prefix}_rank_step_ms_min", med, "min")
        chk.info(f"{prefix}_rank_step_ms_max", med, "max")
    if ms_c:
        med = statistics.median(ms_c)
        chk.info(f"{prefix}_compute_only_rank_ms_min", med, "min")
        chk.info(f"{prefix}_compute_only_rank_ms_max", med, "max")
    b = float(w.bytes_exchanged_per_step())
    chk.info(f"{prefix}_bytes_exchanged_per_step", b, "max")
    chk.info(f"{prefix}_bytes_exchanged_per_step_total", b, "sum")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if os.environ.get("PCMX_STACK_DUMP_S"):  # diagnostic: every rank prints its Python stacks every N seconds
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["PCMX_STACK_DUMP_S"]), repeat=True, file=sys.stderr)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        args.gpus = args.gpus or 1
        if args.gpus > 1:
            return launch(args, argv)
    elif args.gpus is None:  # under a launcher without --gpus: its WORLD_SIZE ranks
        args.gpus = int(world_env)
    elif int(world_env) != args.gpus:  # --gpus given explicitly and different from the launcher's
        print(f"[bench] error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} ranks",
              file=sys.stderr, flush=True)
        return 2

    from parallel_c_programs_amd.models import workloads as W
    from parallel_c_programs_amd.parallel import finalize, init
    from parallel_c_programs_amd.utils.harness import timed
    from parallel_c_programs_amd.utils.metrics import bench_line

    ctx = init(backend=args.backend, device=args.device)
    world, rank, dev = ctx.world, ctx.rank, ctx.device
    if dev.type == "cuda":
        from parallel_c_programs_amd._native import ops as native_ops

        native_ops()  # the HIP extension must load: no silent fallback on a GPU box
        if ctx.backend == "nccl" and world > torch.cuda.device_count():
            raise SystemExit(f"[bench] {world} RCCL ranks but {torch.cuda.device_count()} GPU(s) visible")
    sections = [s for s in args.sections.split(",") if s]
    K, Wm = args.steps, args.warmup
    SETTLE = args.settle_ms
    LIM = W.REL_ERR_LIMIT
    out = {}

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    runner = Runner(ctx, out, args.inject_fault, log)

    # ---- SGEMM (headline value): weak scaling, 8192^3 per GPU
    n = args.size
    head = {"tflops": None, "ms": None}

    def sgemm(chk):
        g = W.Sgemm(ctx, n=n)
        runner.maybe_raise("sgemm", "raise-early")
        yield
        ms, hms = [], []
        t = timed(ctx, g.step, K, Wm, ms, hms, settle_ms=SETTLE)
        rep = g.report(t, K)
        head["tflops"], head["ms"] = rep["value"], rep["ms_per_step"]
        out["sgemm_tflops_per_gpu"] = _r(rep["value"] / world, 3)
        device_times(chk, "sgemm", ms, hms)
        if not args.no_ref and dev.type == "cuda":
            # the vendor library timed exactly like our kernel (same warm-up and step count), into its own buffer:
            # g.c keeps the output of our timed steps for the check
            cref = torch.empty_like(g.c)
            yield
            t_ref = timed(ctx, lambda: torch.matmul(g.a, g.b, out=cref), K, Wm, settle_ms=SETTLE)
            out["hipblaslt_torch_matmul_tflops"] = _r(world * g.work_per_step() * K / t_ref / 1e12, 3)
            del cref
        x6 = not args.no_x6 and dev.type == "cuda" and n % 256 == 0
        if x6:
            # fp32 GEMM on the bf16 matrix cores (exact 3-way operand split, 6 piece products; sgemm_x6.hip): an
            # fp32-accurate extra with its own full fp64 check; never the headline value. Timed before the checks
            # (the checks are local only; every collective of the section comes first)
            gx = W.Sgemm.__new__(W.Sgemm)
            gx.__dict__.update(g.__dict__)
            gx.variant, gx.c = 20, torch.empty_like(g.c)
            yield
            ms6, hms6 = [], []
            t_x6 = timed(ctx, gx.step, K, Wm, ms6, hms6, settle_ms=SETTLE)
            out["sgemm_fp32_via_bf16x6_tflops"] = _r(world * gx.work_per_step() * K / t_x6 / 1e12, 3)
            device_times(chk, "sgemm_fp32_via_bf16x6", ms6, hms6)
        if runner.injected("sgemm", "perturb"):
            g.c[n // 3, n // 5] += 1.0
        yield
        runner.maybe_raise("sgemm")
        chk.error("sgemm_max_rel_err_vs_fp64", g.check(reduce=False)["max_rel_err_vs_fp64"], LIM)
        if x6:
            chk.error("sgemm_fp32_via_bf16x6_max_rel_err_vs_fp64", gx.check(reduce=False)["max_rel_err_vs_fp64"], LIM)
        log(f"sgemm {head['tflops']:.1f} TFLOPS")

    if "sgemm" in sections:
        runner.run("sgemm", sgemm)

    # ---- reduce / scan: weak (rn per GPU) and strong (rn in total); identical runs at N = 1
    rn = int(args.reduce_n)

    def reduce_scan(name, cls, chk):
        for mode, per_rank in (("weak", rn), ("strong", -(-rn // world))):
            if mode == "strong" and world == 1:
                for k in ("gbps", "ms_per_step"):
                    out[f"{name}_strong_{k}"] = out[f"{name}_weak_{k}"]
                v, agg, lim = chk.items[f"{name}_weak_rel_err_vs_fp64"]
                chk.error(f"{name}_strong_rel_err_vs_fp64", v, lim)
                continue
            w = cls(ctx, n=per_rank)
            yield
            ms, hms = [], []
            t = timed(ctx, w.step, K, Wm, ms, hms, settle_ms=SETTLE)
            rep = w.report(t, K)
            out[f"{name}_{mode}_gbps"] = _r(rep["value"], 1)
            out[f"{name}_{mode}_ms_per_step"] = _r(rep["ms_per_step"])
            device_times(chk, f"{name}_{mode}", ms, hms)
            if mode == "weak" and not args.no_ref and dev.type == "cuda":
                # the vendor library on the same per-GPU data, timed exactly like our kernel (rocPRIM behind both)
                yield
                if name == "reduce":
                    t_ref = timed(ctx, lambda: torch.sum(w.x), K, Wm, settle_ms=SETTLE)
                    out["torch_sum_gbps"] = _r(world * 4.0 * w.x.numel() * K / t_ref / 1e9, 1)
                elif ranks_share_gpu(ctx):
                    # rocPRIM's look-back scan waits on blocks by index: with several processes' scans on one GPU
                    # their spinning blocks can hold the CUs the others' predecessors need (seen as a hang at N = 4
                    # on one GPU, profiles/r6_bench/). Our scan takes tiles from a ticket and is safe there.
                    out["torch_cumsum_gbps"] = "not measured: ranks share a GPU"
                else:
                    ybuf = torch.empty_like(w.x)
                    t_ref = timed(ctx, lambda: torch.cumsum(w.x, 0, out=ybuf), K, Wm, settle_ms=SETTLE)
                    out["torch_cumsum_gbps"] = _r(world * 8.0 * w.x.numel() * K / t_ref / 1e9, 1)
                    del ybuf
            if runner.injected(name, "perturb") and mode == "weak":
                if name == "reduce":
                    w.settle()  # (the last timed all-reduce's total stored first, then perturbed)
                    w.total.mul_(1.001)
                else:
                    w.y[w.y.numel() // 3] += 1.0
            yield
            turns = name == "scan" and dev.type == "cuda" and ranks_share_gpu(ctx)
            c = w.check(reduce=False, **({"one_rank_at_a_time": True} if turns else {}))
            chk.error(f"{name}_{mode}_rel_err_vs_fp64", c["rel_err_vs_fp64"], LIM)
            if name == "scan":  # every timed output checked (not a prefix), rank offsets included
                chk.flag(f"scan_{mode}_lookback_ok", c["lookback_ok"])
                prev = chk.items.get("scan_full_max_rel_err_vs_fp64", (0.0,))[0]
                chk.error("scan_full_max_rel_err_vs_fp64", max(prev, c["rel_err_vs_fp64"]), LIM)
            if ctx.distributed:  # the compute-only twin, after the check (it overwrites the checked output)
                yield
                attribute_comm(ctx, chk, out, f"{name}_{mode}", rep["ms_per_step"], ms, w, K, Wm, SETTLE)
            del w
            if dev.type == "cuda":
                torch.cuda.empty_cache()
        runner.maybe_raise(name)  # (after the section's last collective)
        log(f"{name} weak {out[name + '_weak_gbps']} GB/s, strong {out[name + '_strong_gbps']} GB/s")

    for name, cls in (("reduce", W.Reduce), ("scan", W.Scan)):
        if name in sections:
            runner.run(name, lambda chk, name=name, cls=cls: reduce_scan(name, cls, chk))

    # ---- AXPY 1e9 f32 per GPU (the streaming hot loop; weak scaling, no exchange)
    def axpy(chk):
        w = W.Axpy(ctx, n=rn)
        yield
        ms, hms = [], []
        t = timed(ctx, w.step, K, Wm, ms, hms, settle_ms=SETTLE)
        rep = w.report(t, K)
        out["axpy_gbps"], out["axpy_ms_per_step"] = _r(rep["value"], 1), _r(rep["ms_per_step"])
        device_times(chk, "axpy", ms, hms)
        if not args.no_ref and dev.type == "cuda":
            yield
            t_ref = timed(ctx, w.torch_step, K, Wm, settle_ms=SETTLE)
            out["torch_axpy_gbps"] = _r(world * w.work_per_step() * K / t_ref / 1e9, 1)
        if runner.injected("axpy", "perturb"):
            w.y[w.y.numel() // 7] += 1.0
        yield
        c = w.check(reduce=False)
        runner.maybe_raise("axpy")
        chk.error("axpy_rel_err_vs_fp64", c["rel_err_vs_fp64"], LIM)
        out["axpy_steps_checked"] = c["steps_applied"]
        del w
        log(f"axpy {out['axpy_gbps']} GB/s")

    if "axpy" in sections:
        runner.run("axpy", axpy)

    # ---- stencil 16384^2 bf16, strong scaling over row slabs with the overlapped fused halo exchange
    def stencil(chk):
        s = W.Stencil(ctx, n=args.stencil_n, fuse=args.stencil_fuse, halo_mult=args.stencil_halo_mult)
        runner.maybe_raise("stencil", "raise-early")
        yield
        ms, hms = [], []
        t = timed(ctx, s.step, K, Wm, ms, hms, settle_ms=SETTLE)
        rep = s.report(t, K)
        out.update({"stencil_glups": _r(rep["value"], 1), "stencil_ms_per_step": _r(rep["ms_per_step"]),
                    "stencil_updates_per_step": s.slab.fuse, "stencil_halo_mult": s.slab.m})
        device_times(chk, "stencil", ms, hms)
        if runner.injected("stencil", "perturb"):
            s.slab.interior()[s.slab.rows // 2, 7] += 1.0
        yield
        c = s.check(reduce=False)  # (its small-grid distributed run first, then local-only work)
        runner.maybe_raise("stencil")
        out["stencil_timed_grid_updates"] = c["timed_grid_updates"]
        chk.flag("stencil_timed_grid_bit_exact", c["timed_grid_bit_exact"])
        chk.flag("stencil_bit_exact", c["bit_exact_vs_single_step_oracle"])
        chk.flag("stencil_finite", c["finite"])
        if runner.injected("stencil", "selftest"):  # test hook: a deep-halo self-test that failed on this backend
            c["halo_selftest"] = False
        if c["halo_selftest"] is not None:  # the deep halo proven on this backend before timing (N > 1): a failed
            # self-test falls back to m = 1 for the timing but still fails the section (a broken schedule is a bug)
            chk.flag("stencil_halo_selftest_bit_exact", c["halo_selftest"])
        if ctx.distributed:
            yield
            attribute_comm(ctx, chk, out, "stencil", rep["ms_per_step"], ms, s, K, Wm, SETTLE)
        del s
        log(f"stencil {out['stencil_glups']} GLUP/s")

    if "stencil" in sections:
        runner.run("stencil", stencil)

    # ---- SpMV 1e8-nnz power-law graph, strong scaling
    def spmv(chk):
        vendor = not args.no_ref and dev.type == "cuda"
        sp = W.SpMV(ctx, n_rows=int(args.spmv_rows), nnz=int(args.spmv_nnz), chunks=args.spmv_chunks,
                    exchange=args.spmv_exchange, keep_plain=vendor)
        runner.maybe_raise("spmv", "raise-early")
        yield
        ms, hms = [], []
        t = timed(ctx, sp.step, K, Wm, ms, hms, settle_ms=SETTLE)
        rep = sp.report(t, K)
        out.update({"spmv_gflops": _r(rep["value"], 2), "spmv_ms_per_step": _r(rep["ms_per_step"]),
                    "spmv_effective_gbps": _r(rep["effective_gbps"], 1), "spmv_chunks": sp.d.chunks,
                    "spmv_slices": sp.d.slices, "spmv_exchange": sp.d.exchange if ctx.distributed else None,
                    "spmv_colsplit": sp.d.colsplit})
        device_times(chk, "spmv", ms, hms)
        if vendor:  # hipSPARSE (torch sparse CSR x dense vector) on each rank's own rows, the same matrix and x
            yield
            try:
                A = sp.d.vendor_matrix()
                yv = torch.mv(A, sp.xp)
                t_ref = timed(ctx, lambda: torch.mv(A, sp.xp), K, Wm, settle_ms=SETTLE)
                nnz_all = ctx.scalar(float(sp.d.local_nnz))
                ctx.all_reduce_(nnz_all)
                out["torch_sparse_csr_gflops"] = _r(2.0 * nnz_all.item() * K / t_ref / 1e9, 2)
                del A, yv
            except Exception as e:  # the line says so instead of dropping the bar
                out["torch_sparse_csr_gflops"] = f"unsupported on this torch build: {type(e).__name__}: {e}"[:200]
        if runner.injected("spmv", "perturb"):
            sp.y[0] += 1.0
        yield
        c = sp.check(reduce=False)
        chk.error("spmv_max_rel_err_vs_fp64", c["max_rel_err_vs_fp64"], LIM)
        # chained steps x <- A x (the power-iteration pattern, exchanges deferred across step boundaries) vs fp64
        chk.error("spmv_iterated_max_rel_err_vs_fp64", c["iterated_max_rel_err_vs_fp64"], LIM)
        out["spmv_iterated_steps"], out["spmv_deferred_exchange"] = c["iterated_steps"], c["deferred"]
        if runner.injected("spmv", "selftest"):  # test hook: a deferred-pipeline self-test that failed
            c["pipeline_selftest"] = False
        if c["pipeline_selftest"] is not None:  # deferred vs finished-in-step chained steps, bit for bit (N > 1);
            # the timed steps stop deferring on a mismatch, and the section fails
            chk.flag("spmv_pipeline_selftest_bit_identical", c["pipeline_selftest"])
        runner.maybe_raise("spmv")
        if ctx.distributed:
            yield
            attribute_comm(ctx, chk, out, "spmv", rep["ms_per_step"], ms, sp, K, Wm, SETTLE)
            sp.d.finish()
        rows = (sp.d.row0, sp.d.row1)
        del sp
        log(f"spmv {out['spmv_gflops']} GFLOP/s")
        if vendor and world == 1:
            res = rocsparse_bar(int(args.spmv_rows), int(args.spmv_nnz), K, Wm)
            out.update({k: v for k, v in res.items() if not k.startswith("_")})
        elif vendor:
            out.update(rocsparse_bar_ranks(ctx, int(args.spmv_rows), int(args.spmv_nnz), K, Wm, rows))

    if "spmv" in sections:
        runner.run("spmv", spmv)

    # ---- RCCL all-reduce bus bandwidth over xGMI (N > 1)
    def allreduce(chk):
        import torch.distributed as dist

        v = torch.ones(64 << 20, device=dev)
        yield
        kr = max(3, K // 2)
        t_ar = timed(ctx, lambda: dist.all_reduce(v), kr, 1)
        out["allreduce_256MiB_busbw_gbps"] = _r(v.numel() * 4 * 2 * (world - 1) / world * kr / t_ar / 1e9, 1)

    if ctx.distributed and dev.type == "cuda" and ctx.backend == "nccl":
        runner.run("allreduce", allreduce)
    if ctx.distributed:
        import torch.distributed as dist

        from parallel_c_programs_amd.parallel.dist import native_exchange_active

        out["comm_backend"], out["comm_world_size"] = ctx.backend, dist.get_world_size()
        # the per-step exchanges ran on the native RCCL communicator (C++ grouped send / recv), not torch's all_to_all
        out["comm_native_exchange"] = native_exchange_active(ctx)

    rc = 1 if runner.failed else 0
    if rank == 0:
        # BASELINE.json publishes no number ("published": {}), so vs_baseline stays null
        out["checks_passed"] = not runner.failed
        fields = dict(
            metric=METRIC, value=_r(head["tflops"], 3), unit="TFLOPS", n_gpus=world, steps=K, warmup=Wm,
            ms_per_step=_r(head["ms"]), higher_is_better=True, scaling="weak", baseline=None, dtype="fp32",
            data="synthetic (uniform random operands generated on device; power-law CSR generated per rank)",
            config={
                "model": f"SGEMM {n}x{n}x{n} fp32 (v_mfma_f32_32x32x2_f32) per GPU + global reduce/scan "
                         f"{rn:.0e} f32 + stencil {args.stencil_n}^2 bf16 + SpMV {args.spmv_nnz:.0e} nnz",
                "global_batch": world,
                "seq_len": None,
                "parallelism": f"dp{world}",
            },
            device=dev.type, settle_ms_before_warmup=SETTLE if dev.type == "cuda" else 0, **out)
        try:
            line = bench_line(partial="sgemm" not in sections or "sgemm" in runner.failed, **fields)
        except ValueError as e:  # still print what was measured (with the reason), then fail the run after finalize
            line = {k: v for k, v in fields.items() if k != "baseline"}
            line["vs_baseline"] = None
            line["contract_error"], rc = str(e), 1
        print(json.dumps(line), flush=True)
    finalize(ctx)  # every rank reaches this, also when rank 0's line failed the contract
    return rc


if __name__ == "__main__":
    sys.exit(main())
