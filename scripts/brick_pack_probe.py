"""Brick-pack probe for rocprofv3 counter passes: 5 packs of the 512^3 volume + a 1-GiB fill (write-roofline
reference) + a 1-GiB copy."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd._native import ops as native  # noqa: E402

vol = ops.create_volume(512, device="cuda", seed=0)
reg, _ = ops.region3d(vol)
reg = (reg != 0).to(torch.uint8)
for _ in range(5):
    tex = native().brick_pack(vol, reg)
big = torch.empty(1 << 28, device="cuda")
for _ in range(3):
    big.fill_(1.0)
src = torch.empty_like(big)
for _ in range(3):
    big.copy_(src)
torch.cuda.synchronize()
