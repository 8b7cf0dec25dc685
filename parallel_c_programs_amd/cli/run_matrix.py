"""matrix demo (ref 1-introduction/matrix.c:117-225): matrix_t create/print/multiply/resize walkthrough.

--compat reproduces the reference's inverted is_sparse (bug B1) so the printed lines match
the reference binary; the default prints the corrected result."""
from __future__ import annotations

import argparse
import ctypes

from ._common import c_call


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run_matrix")
    ap.add_argument("--compat", action="store_true", help="keep the reference's is_sparse bug (B1)")
    a = ap.parse_args(argv)
    return c_call("pcmx_matrix_demo", ctypes.c_int, [ctypes.c_int], int(a.compat))


if __name__ == "__main__":
    raise SystemExit(main())
