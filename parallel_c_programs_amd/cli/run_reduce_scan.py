"""North-star: global reduction + prefix scan of 1e9 f32 per GPU across ranks (GB/s each)."""
import sys

from .run_workload import run


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    run("reduce", argv, {"n": 10**9})
    run("scan", argv, {"n": 10**9})
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
