"""Distributed 3-D pipeline over z-slabs (SURVEY C9 "optional z-slab split across GPUs"): one process per GPU,
launched with torch.distributed.run (gloo on CPU). Every rank generates its own planes of the dim^3 volume,
the ranks grow the region from the reference seed (50, 300, 300) with halo-plane exchange, then ray-cast it
with the pipelined slab caster (bit-identical to the single-volume reference caster); rank 0 writes ./out.bmp
and prints one JSON line (region voxels, outer steps, host reads, grow / raycast seconds).

  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
         -m parallel_c_programs_amd.cli.run_volume3d --dim 512 --image-dim 512
"""
from __future__ import annotations

import argparse
import json
import time

import torch

from ..parallel import DistributedVolume, finalize, init
from ..utils import bmp


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run_volume3d")
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--image-dim", type=int, default=512)
    ap.add_argument("--backend", default=None)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    ctx = init(a.backend, a.device)
    try:
        def sync():
            if ctx.device.type == "cuda":
                torch.cuda.synchronize(ctx.device)
            ctx.barrier()

        dv = DistributedVolume(ctx, a.dim)
        sync()
        t0 = time.perf_counter()
        n = torch.tensor([dv.grow()], dtype=torch.int64, device=ctx.device)
        sync()
        t1 = time.perf_counter()
        img = dv.raycast(a.image_dim)
        sync()
        t2 = time.perf_counter()
        ctx.all_reduce_(n)
        if ctx.is_root:
            bmp.write_out_bmp(img.cpu().numpy())
            print(json.dumps({"workload": "volume3d_zslabs", "n_ranks": ctx.world, "dim": a.dim,
                              "image_dim": a.image_dim, "region_voxels": int(n.item()), **dv.stats,
                              "grow_s": round(t1 - t0, 6), "raycast_s": round(t2 - t1, 6),
                              "image_sum": int(img.long().sum())}), flush=True)
    finally:
        finalize(ctx)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
