"""North-star: CSR SpMV on a 1e8-nnz power-law graph, nnz-balanced over ranks + all-gather (GFLOP/s)."""
from .run_workload import run


def main(argv=None) -> int:
    run("spmv", argv, {"n_rows": 10_000_000, "nnz": 100_000_000})
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
