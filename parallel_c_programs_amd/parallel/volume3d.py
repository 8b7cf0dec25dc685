"""Z-slab decomposition of the 3-D pipeline over ranks (SURVEY C9 "optional z-slab split across GPUs"; ancestors:
the single-GPU pipeline of ref 5-cuda-region-growing/raycast.cu:702-822 and the halo-exchange fixpoint loop of
ref 2-mpi-region-growing/region.c:493-533).

Each rank owns planes [z0, z1) of the dim^3 volume and keeps them in (nz + 2, dim, dim) buffers whose first and
last planes are halos (global planes z0 - 1 and z1). Nothing is ever assembled on one device: a 4096^3 volume
(64 GB of data + region) spreads over the 288 GB HBM of the ranks.

  * volume   every rank generates its own planes (+ halos) with the deterministic hash volume (same bytes as
             the single-device generator), on the GPU or the host.
  * grow     region growing from the reference seed (50, 300, 300): the local step is the bit-parallel tiled
             grower on the slab (halo planes are read-only seeds; csrc/kernels/region.hip grow_slab), then the
             two boundary planes go to the z-neighbours in one grouped send/recv and land in their halo planes.
             Termination is device-resident: a "halo changed" flag is raised on the device, MAX-all-reduced in
             place and read by the host once every CHECK_EVERY outer steps (as parallel/region2d.py).
  * raycast  the reference caster (f64 colour update, bit-exact with the serial caster) as a pipeline of slab
             stages: the rays of the reference camera run towards -z, so the top slab marches first from the
             camera and hands every pixel's state {position, colour, steps, flags} to the slab below, which
             resumes exactly where the ray left (same float position sequence); the bottom slab writes the image.
             The image is bit-identical to the single-volume caster. (Stages are sequential per frame; frames can
             overlap across stages.)
"""
from __future__ import annotations

import ctypes

import torch

from .._native import cpu_lib
from .._native import ops as native
from ..ops.image import SEED_3D, default_camera
from .dist import Context
from .topology import split

CHECK_EVERY = 2  # outer grow steps per host read of the all-reduced "halo changed" flag


class VolumeSlab:
    """Planes [z0, z1) of a dim^3 volume (+ one halo plane each side) on `device`."""

    def __init__(self, dim: int, z0: int, z1: int, device, seed: int = 0):
        self.dim, self.z0, self.z1, self.nz = dim, z0, z1, z1 - z0
        self.device = torch.device(device)
        self.data = torch.empty((self.nz + 2, dim, dim), dtype=torch.uint8, device=self.device)
        if self.device.type == "cuda":
            native().volume_gen_slab_(self.data, z0 - 1, seed)
        else:
            cpu_lib().pcmx_create_data_hash_slab(ctypes.c_void_p(self.data.data_ptr()), dim, z0 - 1, self.nz + 2,
                                                 ctypes.c_uint(seed))
        self.region = torch.zeros_like(self.data)

    # ---- region growing
    def seed(self, xyz=SEED_3D) -> None:
        x, y, z = xyz
        if self.z0 <= z < self.z1:
            self.region[z - self.z0 + 1, y, x] = 1

    def grow_local(self, halos: int, threshold: int = 1) -> int:
        """Local fixpoint over the owned planes; halo planes (halos bit 0 below, bit 1 above) are seeds only."""
        if self.device.type == "cuda":
            return int(native().region3d_grow_slab_(self.region, self.data, halos, threshold))
        P = self.dim * self.dim
        lib = cpu_lib()
        lib.pcmx_region3d_slab_host.restype = ctypes.c_longlong
        lib.pcmx_region3d_slab_host(ctypes.c_void_p(self.data.data_ptr() + P), ctypes.c_void_p(self.region.data_ptr() + P),
                                    self.dim, self.nz, halos, threshold)
        return 0

    def owned_region(self) -> torch.Tensor:
        return self.region[1:self.nz + 1]

    # ---- ray casting
    def raycast_stage(self, state: torch.Tensor, init: bool, bottom: bool, image_dim: int) -> torch.Tensor | None:
        cam = default_camera(image_dim)
        if self.device.type == "cuda":
            img = native().raycast_slab_(self.data, (self.region != 0).to(torch.uint8), self.z0, state, init, bottom,
                                         image_dim, cam.cam12(), float(cam.pixel_width), float(cam.step_size),
                                         int(cam.max_steps))
            return img if bottom else None
        img = torch.empty((image_dim, image_dim), dtype=torch.uint8) if bottom else None
        reg = (self.region != 0).to(torch.uint8).contiguous()
        cpu_lib().pcmx_raycast_slab_host(ctypes.c_void_p(self.data.data_ptr()), ctypes.c_void_p(reg.data_ptr()),
                                         self.dim, self.z0, self.z1, image_dim, ctypes.c_void_p(state.data_ptr()),
                                         int(init), int(bottom), ctypes.c_void_p(img.data_ptr() if bottom else 0))
        return img


class DistributedVolume:
    """One rank's slab of the distributed 3-D pipeline (rank r owns planes split(dim, world, r))."""

    def __init__(self, ctx: Context, dim: int = 512, seed: int = 0):
        self.ctx = ctx
        z0, z1 = split(dim, ctx.world, ctx.rank)
        if z1 - z0 < 1:
            raise ValueError("every rank needs at least one plane")
        self.slab = VolumeSlab(dim, z0, z1, ctx.device, seed)
        self.below = ctx.rank - 1 if ctx.rank > 0 else -1  # owner of plane z0 - 1
        self.above = ctx.rank + 1 if ctx.rank < ctx.world - 1 else -1  # owner of plane z1
        self.halos = (1 if self.below >= 0 else 0) | (2 if self.above >= 0 else 0)
        self.stats: dict = {}

    def _exchange(self, changed: torch.Tensor) -> None:
        """Boundary planes to the z-neighbours (one grouped send/recv), landing in their halo planes; raises
        `changed` on the device when a halo plane takes new values."""
        s, nz = self.slab, self.slab.nz
        pairs, recv = [], []
        if self.below >= 0:
            buf = torch.empty_like(s.region[0])
            pairs.append((self.below, s.region[1].contiguous(), buf))
            recv.append((0, buf))
        if self.above >= 0:
            buf = torch.empty_like(s.region[0])
            pairs.append((self.above, s.region[nz].contiguous(), buf))
            recv.append((nz + 1, buf))
        self.ctx.neighbour_exchange(pairs)  # one RCCL call (Context.neighbour_exchange)
        for plane, buf in recv:
            changed.logical_or_(torch.ne(s.region[plane], buf).any().reshape(1))
            s.region[plane].copy_(buf)

    def grow(self, threshold: int = 1, xyz=SEED_3D) -> int:
        """Distributed region growing; returns this rank's region voxel count."""
        s, ctx = self.slab, self.ctx
        s.region.zero_()
        s.seed(xyz)
        changed = torch.zeros(1, dtype=torch.bool, device=s.device)
        flag = torch.zeros(1, dtype=torch.int32, device=s.device)
        outer = reads = launches = 0
        while True:
            launches += s.grow_local(self.halos, threshold)
            outer += 1
            if not ctx.distributed:
                break
            self._exchange(changed)
            if outer % CHECK_EVERY:
                continue
            flag.copy_(changed)
            ctx.all_reduce_(flag, "max")
            reads += 1
            if int(flag.item()) == 0:  # the loop's only host read-back
                break
            changed.zero_()
        self.stats = {"outer_steps": outer, "host_reads": reads, "launches": launches}
        return int((s.owned_region() != 0).sum())

    def raycast(self, image_dim: int = 512) -> torch.Tensor | None:
        """Pipelined slab caster; returns the image on rank 0 (the bottom slab), None elsewhere."""
        s, ctx = self.slab, self.ctx
        state = torch.zeros((image_dim * image_dim, 6), dtype=torch.int32, device=s.device)
        top = self.above < 0
        if not top:
            ctx.recv(state, self.above)
        img = s.raycast_stage(state, init=top, bottom=self.below < 0, image_dim=image_dim)
        if self.below >= 0:
            ctx.send(state, self.below)
        return img

    def gather_region(self) -> torch.Tensor | None:
        """The full (dim, dim, dim) region on rank 0 (tests and small volumes only)."""
        s, ctx = self.slab, self.ctx
        mine = (s.owned_region() != 0).to(torch.uint8).contiguous()
        if not ctx.distributed:
            return mine
        if ctx.is_root:
            parts = [mine]
            for r in range(1, ctx.world):
                a, b = split(s.dim, ctx.world, r)
                buf = torch.empty((b - a, s.dim, s.dim), dtype=torch.uint8, device=s.device)
                ctx.recv(buf, r)
                parts.append(buf)
            return torch.cat(parts)
        ctx.send(mine, 0)
        return None


def emulate_slabs(dim: int, parts: int, device, seed: int = 0, threshold: int = 1, image_dim: int = 64):
    """All slab stages of a `parts`-rank decomposition run in ONE process on one device (the multi-rank device
    path exercised on a single GPU): returns (region volume, image, outer steps)."""
    slabs = [VolumeSlab(dim, *split(dim, parts, r), device, seed) for r in range(parts)]
    for s in slabs:
        s.seed()
    outer = 0
    while True:
        for k, s in enumerate(slabs):
            s.grow_local((1 if k > 0 else 0) | (2 if k < parts - 1 else 0), threshold)
        outer += 1
        changed = False
        for k in range(parts - 1):  # plane exchange between slab k (below) and k + 1 (above)
            lo, hi = slabs[k], slabs[k + 1]
            top_of_lo, bottom_of_hi = lo.region[lo.nz].clone(), hi.region[1].clone()
            changed |= not torch.equal(hi.region[0], top_of_lo) or not torch.equal(lo.region[lo.nz + 1], bottom_of_hi)
            hi.region[0].copy_(top_of_lo)
            lo.region[lo.nz + 1].copy_(bottom_of_hi)
        if not changed or parts == 1:
            break
    region = torch.cat([(s.owned_region() != 0).to(torch.uint8) for s in slabs])
    state = torch.zeros((image_dim * image_dim, 6), dtype=torch.int32, device=slabs[0].device)
    img = None
    for k in range(parts - 1, -1, -1):
        img = slabs[k].raycast_stage(state, init=k == parts - 1, bottom=k == 0, image_dim=image_dim)
    return region, img, outer
