"""Histogram equalisation (ref 4-histogram-equalization-openmp-pthreads): `run_histogram image n_threads`.

--method serial|omp|pthreads runs the host C implementations (identical output to the reference programs
histogram_serial / _omp / _pthreads); --method gpu runs the fused gfx950 kernel. Writes ./out.bmp."""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

from ._common import c_call

METHODS = {"serial": 0, "omp": 1, "pthreads": 2}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    pos = [x for x in argv if not x.startswith("--")]
    if len(pos) < 2:
        print("Useage: run_histogram image n_threads", flush=True)
        return 255
    ap = argparse.ArgumentParser(prog="run_histogram")
    ap.add_argument("image")
    ap.add_argument("n_threads", type=int)
    ap.add_argument("--method", default="serial", choices=[*METHODS, "gpu"])
    a = ap.parse_args(argv)
    if a.method != "gpu":
        return c_call("pcmx_histogram_demo", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int],
                      os.fsencode(a.image), a.n_threads, METHODS[a.method])
    import numpy as np
    import torch

    from .. import ops
    from ..utils import bmp

    img = torch.from_numpy(bmp.read(a.image)).cuda()
    bmp.write_out_bmp(np.ascontiguousarray(ops.histeq(img).cpu().numpy()))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
