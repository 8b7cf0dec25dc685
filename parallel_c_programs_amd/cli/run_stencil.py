"""North-star: 5-point stencil on a 16384^2 bf16 grid, row slabs + overlapped halo exchange (GLUP/s)."""
from .run_workload import run


def main(argv=None) -> int:
    run("stencil", argv, {"n": 16384})
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
