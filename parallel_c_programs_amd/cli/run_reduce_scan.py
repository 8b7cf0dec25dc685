"""North-star reduce / scan CLI: global sum and global inclusive prefix sum of N f32 per GPU (default 1e9, weak
scaling) across the ranks (GB/s). Reduce: local HBM reduction + one-scalar RCCL all-reduce. Scan: local sums, an
exclusive scan of them across the ranks, then the single-pass look-back scan seeded with the rank's offset.
Ancestor: MPI_Allreduce of the distributed region growing, ref 2-mpi-region-growing/region.c:435-440.

    run_reduce_scan [N] [--op reduce|scan|both] [--steps S --warmup W] [--no-check]

Each op prints the reference's "Time : %f s" line and one JSON line (the check: fp64 reference; the scan check
covers every output of every rank)."""
import sys

from .run_workload import run


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    ops = ["reduce", "scan"]
    if "--op" in argv:
        i = argv.index("--op")
        op = argv[i + 1] if i + 1 < len(argv) else ""
        if op not in ("reduce", "scan", "both"):
            print("run_reduce_scan: --op reduce|scan|both", file=sys.stderr)
            return 2
        ops = ["reduce", "scan"] if op == "both" else [op]
        del argv[i:i + 2]

    def _args(ap):
        ap.add_argument("n", nargs="?", type=float, default=1e9, help="f32 elements per GPU")

    for name in ops:
        run(name, argv, {"n": 10**9}, _args, lambda a: {"n": int(a.n)}, prog="run_reduce_scan", doc=__doc__,
            time_line=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
