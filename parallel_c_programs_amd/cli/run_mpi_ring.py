"""Token chain (ref 1-introduction/mpi.c). Launch:
    python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 -m parallel_c_programs_amd.cli.run_mpi_ring
"""
from __future__ import annotations

import argparse

from ..parallel import finalize, init, token_ring


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run_mpi_ring")
    ap.add_argument("--backend", default=None, help="nccl (RCCL) | gloo")
    a = ap.parse_args(argv)
    ctx = init(a.backend, "cpu" if a.backend == "gloo" else None)
    try:
        token_ring(ctx)
    finally:
        finalize(ctx)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
