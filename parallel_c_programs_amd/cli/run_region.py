"""Distributed 2-D region growing (ref 2-mpi-region-growing/region.c).

    python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 \
        -m parallel_c_programs_amd.cli.run_region pic1.bmp

Same argv and output as `mpirun -n P region pic1.bmp`: root writes ./out.bmp = image * (region == 0).
Extra flags: --threshold, --dims R C (process grid), --backend, --stats (timing + step counts on stderr).
Any P works (the reference only handled square grids, B8)."""
from __future__ import annotations

import argparse
import sys
import time

import numpy as np
import torch

from ..ops.image import apply_region_mask
from ..parallel import finalize, grow_distributed, init
from ..utils import bmp


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    pos = [a for a in argv if not a.startswith("--")]
    if len(pos) < 1:
        print("Useage: region file", end="", flush=True)  # ref region.c:553 (no newline, B12)
        return 255
    ap = argparse.ArgumentParser(prog="run_region")
    ap.add_argument("file")
    ap.add_argument("--threshold", type=int, default=2)
    ap.add_argument("--dims", type=int, nargs=2, default=None)
    ap.add_argument("--backend", default=None)
    ap.add_argument("--device", default=None, help="cpu or cuda (default: cpu with --backend gloo, else the GPU)")
    ap.add_argument("--out", default="out.bmp")
    ap.add_argument("--stats", action="store_true")
    a = ap.parse_args(argv)
    ctx = init(a.backend, a.device or ("cpu" if a.backend == "gloo" else None))
    try:
        image = torch.from_numpy(bmp.read(a.file)) if ctx.is_root else None
        stats: dict = {}
        ctx.barrier()
        t0 = time.perf_counter()
        region = grow_distributed(ctx, image, a.threshold, dims=tuple(a.dims) if a.dims else None, stats=stats)
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if ctx.is_root:
            out = apply_region_mask(image, region.cpu())
            bmp.write(a.out, np.ascontiguousarray(out.numpy()))
            if a.stats:
                print(f"ranks={ctx.world} dims={stats['dims']} outer_steps={stats['outer_steps']} "
                      f"launches={stats['launches']} region={int(region.sum())} time={dt:.6f}s", file=sys.stderr)
    finally:
        finalize(ctx)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
