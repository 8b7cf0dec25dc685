"""North-star SpMV CLI: y = A x on a synthetic power-law CSR graph (default 1e7 rows, 1e8 nnz), rows partitioned by
nnz over the ranks, x entries exchanged as ghosts (GFLOP/s). Ancestor: the CSR benchmark of
ref 3-serial-optimization/spmv.c:170-177, 331-367.

    run_spmv_dist [ROWS] [NNZ] [--alpha A] [--chunks C] [--slices S] [--exchange ghost|allgather] [--steps S ...]

  --chunks C     exchange pipeline depth (default 1 at N = 1, 2 above): chunk c's exchange overlaps chunk c+1's product
  --slices S     XCD column slices of the product kernel (0: plain CSR-adaptive; default by vector length)
  --exchange     ghost (only the x entries each rank's rows reference) or allgather (the whole vector)

The check compares every rank's rows (and every ghost it received) with an fp64 product."""
from .run_workload import run


def _args(ap):
    ap.add_argument("rows", nargs="?", type=float, default=1e7)
    ap.add_argument("nnz", nargs="?", type=float, default=1e8)
    ap.add_argument("--alpha", type=float, default=None, help="power-law exponent of the row degrees (2.5)")
    ap.add_argument("--chunks", type=int, default=None)
    ap.add_argument("--slices", type=int, default=None)
    ap.add_argument("--exchange", choices=("ghost", "allgather"), default=None)


def _cfg(a):
    return {"n_rows": int(a.rows), "nnz": int(a.nnz), "alpha": a.alpha, "chunks": a.chunks, "slices": a.slices,
            "exchange": a.exchange}


def main(argv=None) -> int:
    run("spmv", argv, {"n_rows": 10_000_000, "nnz": 100_000_000}, _args, _cfg, doc=__doc__, time_line=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
