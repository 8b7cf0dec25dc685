"""3-D region growing + volume ray casting (ref 5-cuda-region-growing/raycast.cu:824-854, SURVEY §3.2;
OpenCL variant ref 6-opencl-region-growing/raycast.c:439-448).

Default = the CUDA program: device info, 512^3 volume, LDS-tiled region growing from (50,300,300),
"Grow time:", texture-path ray cast, "Raycast time:", 512x512 ./out.bmp.
--opencl = the OpenCL program's choices: naive (one sweep per launch) region kernel, global-memory caster,
64x64 image. --volume rand uses the reference's exact rand() volume (host generated); the default "hash"
volume is generated on the GPU."""
from __future__ import annotations

import argparse
import time

import numpy as np
import torch

from .. import ops
from ..utils import bmp
from ..utils.device import print_device_info
from ..utils.timing import print_time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run_raycast")
    ap.add_argument("--opencl", action="store_true", help="OpenCL variant: naive grow, global caster, 64^2")
    ap.add_argument("--image-dim", type=int, default=None)
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--grow", choices=["tiled", "naive"], default=None)
    ap.add_argument("--cast", choices=["texture", "global", "global_f32"], default=None)
    ap.add_argument("--volume", choices=["hash", "rand"], default="hash")
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    dev = torch.device(a.device or ("cuda" if torch.cuda.is_available() else "cpu"))
    image_dim = a.image_dim or (64 if a.opencl else 512)
    grow = a.grow or ("naive" if a.opencl else "tiled")
    cast = a.cast or ("global" if a.opencl else "texture")
    if dev.type == "cpu":
        cast = "global"
    if not a.opencl and dev.type == "cuda":
        print_device_info(dev.index or 0)
    data = ops.create_volume(a.dim, device=dev, background=a.volume)

    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    region, launches = ops.region3d(data, method=grow)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    if not a.opencl:
        print("\nGrow time:")
        print_time(t1 - t0)
        print("Errors: no error", flush=True)

    t0 = time.perf_counter()
    image = ops.raycast(data, (region > 0).to(torch.uint8), image_dim, method=cast)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    if not a.opencl:
        print("\nRaycast time: ")
        print_time(t1 - t0)
        print("Errors: no error", flush=True)
    bmp.write_out_bmp(np.ascontiguousarray(image.cpu().numpy()))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
