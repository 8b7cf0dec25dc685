"""North-star: SGEMM 8192^2 fp32 on the MFMA kernel (TFLOPS). Flags as run_workload; e.g. --set n=4096."""
from .run_workload import run


def main(argv=None) -> int:
    run("sgemm", argv, {"n": 8192})
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
