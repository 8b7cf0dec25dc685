"""Ray-cast lab: time the texture ray marcher (brick-packed volume) at each segment split and prefetch batch size,
512^2 image.
Usage: python scripts/raycast_lab.py"""
import sys

import torch

sys.path.insert(0, ".")
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd._native import ops as native  # noqa: E402
from parallel_c_programs_amd.ops.image import default_camera  # noqa: E402

vol = ops.create_volume(512, device="cuda", seed=0)
reg, _ = ops.region3d(vol, threshold=1)
tex = native().brick_pack(vol, (reg != 0).to(torch.uint8))

cam = default_camera(512)


def run(max_steps=None, batch=0, segments=0):
    return native().raycast_bricked(tex, 512, cam.cam12(), float(cam.pixel_width), float(cam.step_size),
                                    int(max_steps or cam.max_steps), batch, segments)


def timeit(fn, reps=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


regb = (reg != 0).to(torch.uint8)
print(f"brick_pack (narrow 8-B texels): {timeit(lambda: native().brick_pack(vol, regb)):.3f} ms")
print(f"brick_pack (wide 16-B texels, data | 128): {timeit(lambda: native().brick_pack(vol | 128, regb)):.3f} ms")
for ms in (1000, 2000, 3000, 4000, 5000):
    print(f"max_steps {ms}: {timeit(lambda: run(ms)):.3f} ms")




ref = None
for rnd in range(2):
    for b, seg in ((4, 1), (16, 1), (16, 2), (8, 4), (16, 4)):
        img = run(batch=b, segments=seg)
        ms = timeit(lambda: run(batch=b, segments=seg))
        ref = img if ref is None else ref
        diff = (img.float() - ref.float()).abs()
        print(f"batch {b:2d} segments {seg}: {ms:.3f} ms  max|diff| vs batch 4 x 1 segment {diff.max().item():.0f}  "
              f"pixels differing {int((diff > 0).sum())}", flush=True)
