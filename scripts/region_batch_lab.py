"""Region-growing lab: launches per pipelined fixpoint batch (3-D tiled grower on the 512^3 reference volume,
2-D grower on pic1.bmp). Each batch's changed-flag check overlaps the next batch; after convergence one
speculative batch of no-op launches runs, so the batch size trades that tail against check overhead.
usage: python scripts/region_batch_lab.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd._native import ops as native  # noqa: E402
from parallel_c_programs_amd.ops.image import SEED_3D  # noqa: E402
from parallel_c_programs_amd.utils.timing import device_time_ms  # noqa: E402

vol = ops.create_volume(512, device="cuda", seed=0)
x, y, z = SEED_3D
reg = torch.zeros_like(vol)


def grow3(batch):
    reg.zero_()
    reg[z, y, x] = 1
    return native().region3d_grow_(reg, vol, 1, True, batch, 1_000_000)


for rnd in range(2):
    for b in (2, 4, 8, 16):
        n = grow3(b)
        ms = device_time_ms(lambda: grow3(b), reps=10, warmup=2)
        print(f"3-D batch {b:2d}: {ms:.3f} ms per grow (incl. zero + seed), {n} launches, "
              f"{int((reg != 0).sum())} voxels", flush=True)
