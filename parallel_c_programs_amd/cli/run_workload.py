"""Generic north-star driver: `run_workload <name> [--steps K] [--warmup W] [--set key=value ...]`.

One process per GPU (launch with torch.distributed.run for N > 1); prints one JSON line on rank 0 with the
whole-job throughput (sum over ranks), the max-over-ranks step time and the workload's numerics check."""
from __future__ import annotations

import argparse
import sys

from ..models import WORKLOADS, build_workload
from ..parallel import finalize, init
from ..utils.harness import timed
from ..utils.metrics import emit_metric
from ..utils.timing import print_time


def _val(s: str):
    for cast in (int, float):
        try:
            return cast(s)
        except ValueError:
            pass
    return {"true": True, "false": False}.get(s.lower(), s)


class CheckFailed(SystemExit):
    """The workload's numerics check failed: its JSON line is printed, then the process exits 1."""


def run(name: str, argv=None, defaults: dict | None = None, add_args=None, to_cfg=None, prog: str | None = None,
        doc: str | None = None, time_line: bool = False) -> dict | None:
    """Builds workload `name` from defaults <- to_cfg(parsed CLI args) <- --set key=value, times it like bench.py
    (warm-up, then `steps` steps between barrier + device syncs, max over ranks) and prints one JSON line on rank 0
    (preceded by the reference's "Time : %f s" per step when time_line). A failed numerics check ("check_passed"
    false in the line) exits the process with status 1 after the line is printed (CheckFailed)."""
    ap = argparse.ArgumentParser(prog=prog or f"run_{name}", description=doc,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    if add_args:
        add_args(ap)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--backend", default=None, help="nccl (RCCL, default on a GPU) or gloo")
    ap.add_argument("--device", default=None, help="cuda (default with a GPU) or cpu")
    ap.add_argument("--no-check", action="store_true", help="skip the workload's numerics check")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE", help="any workload config key")
    a = ap.parse_args(argv)
    cfg = dict(defaults or {})
    if to_cfg:
        cfg.update({k: v for k, v in to_cfg(a).items() if v is not None})
    cfg.update({k: _val(v) for k, v in (s.split("=", 1) for s in a.set)})
    ctx = init(a.backend, a.device)
    try:
        w = build_workload(name, ctx, **cfg)
        secs = timed(ctx, w.step, a.steps, a.warmup)
        rep = w.report(secs, a.steps)
        chk = {} if a.no_check else w.check()
        out = {"workload": name, "n_ranks": ctx.world, "device": ctx.device.type, "steps": a.steps,
               "warmup": a.warmup, "config": w.cfg, **{k: (round(v, 4) if isinstance(v, float) else v)
                                                       for k, v in rep.items()}, **chk}
        if ctx.is_root:
            if time_line:
                print_time(rep["ms_per_step"] / 1e3)
            emit_metric(**out)
    finally:
        finalize(ctx)
    if not out.get("check_passed", True):
        raise CheckFailed(1)
    return out


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in WORKLOADS:
        print(f"usage: run_workload {{{'|'.join(WORKLOADS)}}} [--steps K] [--warmup W] [--set k=v]")
        return 2
    run(argv[0], argv[1:])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
