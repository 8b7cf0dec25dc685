"""Reference-algorithm 3-D kernels on one MI355X (round 5, against the reference's own OpenCL program run on the same
GPU: profiles/r5_refbase/): the global-memory ray caster's variants (0: production, the samples of 8 steps in flight on
8x8-pixel one-wave tiles; 1: round 4, one step in flight on 16x16 tiles; 2 / 3: 4 / 16 steps in flight) at 64^2 (the
OpenCL program) and 512^2, every image checked against variant 1 bit for bit; and the naive 0/1/2 frontier grower
(one launch per BFS level, the reference's algorithm) against the tiled grower. Prints ms per call (events).
usage: python scripts/raycast_global_lab.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
# round 6: 4 = batch caster with pair taps, 5 / 6 / 7 / 8 = group-per-ray caster with 64 / 16 / 8 / 4 lanes per ray
VARIANTS = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 0, 2, 3, 1, 0]
GROW = len(sys.argv) <= 3 or sys.argv[3] != "nogrow"
dev = torch.device("cuda", 0)


def timed(fn, n=reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        out = fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n, out


vol = ops.create_volume(512, device=dev, seed=0)
for method in (("naive", "tiled", "naive", "tiled") if GROW else ("tiled",)):
    ms, (reg, launches) = timed(lambda: ops.region3d(vol, threshold=1, method=method))
    print(f"grow {method:5s} {ms:8.3f} ms per grow ({launches} launches)  voxels {int((reg != 0).sum())}", flush=True)
region = (reg != 0).to(torch.uint8)
for image_dim in (64, 512):
    ref = ops.raycast(vol, region, image_dim, method="global", variant=1)
    for v in VARIANTS:
        ms, img = timed(lambda: ops.raycast(vol, region, image_dim, method="global", variant=v))
        print(f"raycast global {image_dim:3d}^2 variant {v}: {ms:8.3f} ms  sum {int(img.long().sum())}"
              f"{'' if torch.equal(img, ref) else '  MISMATCH'}", flush=True)
    ref32 = ops.raycast(vol, region, image_dim, method="global_f32", variant=1)
    for v in sorted(set(VARIANTS)):
        ms, img = timed(lambda: ops.raycast(vol, region, image_dim, method="global_f32", variant=v))
        print(f"raycast global_f32 {image_dim:3d}^2 variant {v}: {ms:8.3f} ms  sum {int(img.long().sum())}"
              f"{'' if torch.equal(img, ref32) else '  MISMATCH'}", flush=True)
    ms, img = timed(lambda: ops.raycast(vol, region, image_dim, method="texture"))
    print(f"raycast texture {image_dim:3d}^2: {ms:8.3f} ms (pack + march)", flush=True)
