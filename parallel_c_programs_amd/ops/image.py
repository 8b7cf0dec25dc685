"""Image / volume ops: histogram equalisation, 2-D and 3-D region growing, volume generation, ray casting.

Reference parity (anonyomous4/parallel-c-programs):
  histeq          4-histogram-equalization-openmp-pthreads/histogram_serial.c:11-42 (+ _omp.c, _pthreads.c)
  region2d        2-mpi-region-growing/region.c:493-533 (4-connected, |a-b| < 2, seeded flood fill)
  region3d        5-cuda-region-growing/raycast.cu:534-822 (naive + shared-memory kernels, 6-connected)
  volume          5-cuda-region-growing/raycast.cu:114-158 (create_data)
  raycast         5-cuda-region-growing/raycast.cu:216-531, 6-opencl-region-growing/raycast.cl:93-137
GPU tensors run the gfx950 kernels; CPU tensors run the host C library (serial oracles / OpenMP).
"""
from __future__ import annotations

import ctypes

import torch

from .._native import cpu_lib, ops

# ------------------------------------------------------------------------------- histogram equalisation


def histeq(img: torch.Tensor, method: str = "auto", n_threads: int = 4) -> torch.Tensor:
    """Equalise an 8-bit image (bit-identical to the serial reference on every path).

    method (CPU only): "serial" | "omp" | "pthreads". GPU tensors always run the two-launch gfx950 path
    (per-lane LDS counters + bank-replicated LUT map, csrc/kernels/histeq.hip); "auto" / "multiblock" are
    accepted for GPU tensors.
    """
    if img.dtype != torch.uint8:
        raise TypeError("histeq: uint8 image expected")
    if img.is_cuda:
        if method not in ("auto", "multiblock"):
            raise ValueError(f"histeq: method {method!r} is CPU-only")
        return ops().histeq(img.contiguous()).view(img.shape)
    src = img.contiguous()
    out = torch.empty_like(src)
    lib = cpu_lib()
    if method in ("auto", "serial"):
        lib.pcmx_histeq_serial(src.data_ptr(), out.data_ptr(), src.numel())
    elif method == "omp":
        lib.pcmx_histeq_omp(src.data_ptr(), out.data_ptr(), src.numel(), n_threads)
    elif method == "pthreads":
        lib.pcmx_histeq_pthreads(src.data_ptr(), out.data_ptr(), src.numel(), n_threads)
    else:
        raise ValueError(f"unknown histeq method {method!r}")
    return out


# ------------------------------------------------------------------------------- region growing 2-D

DEFAULT_SEED_OFFSET = 5  # ref region.c:451 seed_pos, in 1-padded coordinates


def corner_seeds(h: int, w: int, offset: int = DEFAULT_SEED_OFFSET) -> list[tuple[int, int]]:
    """The reference's four corner seeds (ref region.c:450-490) as unpadded (x, y)."""
    o = offset - 1
    return [(o, o), (w - offset - 1, o), (w - offset - 1, h - offset - 1), (o, h - offset - 1)]


def pad1(t: torch.Tensor, value: int = 0) -> torch.Tensor:
    """(H, W) -> (H+2, W+2) with a constant 1-cell ring (the tile + halo layout)."""
    return torch.nn.functional.pad(t.unsqueeze(0), (1, 1, 1, 1), value=value).squeeze(0).contiguous()


def region2d_grow_padded_(region_p: torch.Tensor, img_p: torch.Tensor, threshold: int = 2, batch: int = 4,
                          max_launches: int = 100000) -> int:
    """Grow `region_p` in place on padded (H+2, W+2) uint8 tensors; halo cells are read-only seeds.

    Returns the number of kernel launches (GPU) or 0 (CPU). The distributed driver calls this per rank.
    """
    if region_p.is_cuda:
        return int(ops().region2d_grow_(region_p, img_p, int(threshold), int(batch), int(max_launches)))
    _region2d_padded_cpu(region_p, img_p, threshold)
    return 0


def _region2d_padded_cpu(region_p: torch.Tensor, img_p: torch.Tensor, threshold: int) -> None:
    # host path: seeds = interior region pixels + halo region pixels; grow inside the interior only
    H, W = img_p.shape[0] - 2, img_p.shape[1] - 2
    reg = region_p.numpy() if region_p.is_contiguous() else region_p.contiguous().numpy()
    img = img_p.numpy().astype("int32")
    import numpy as np

    stack = list(zip(*np.nonzero(reg)))
    while stack:
        y, x = stack.pop()
        v = img[y, x]
        for dy, dx in ((1, 0), (-1, 0), (0, 1), (0, -1)):
            ny, nx = y + dy, x + dx
            if 1 <= ny <= H and 1 <= nx <= W and not reg[ny, nx] and abs(int(img[ny, nx]) - int(v)) < threshold:
                reg[ny, nx] = 1
                stack.append((ny, nx))
    if not region_p.is_contiguous():
        region_p.copy_(torch.from_numpy(reg))


def region2d(img: torch.Tensor, seeds=None, threshold: int = 2) -> torch.Tensor:
    """Region bitmap (uint8 0/1) of a seeded 4-connected flood fill with |a-b| < threshold."""
    if img.dtype != torch.uint8 or img.dim() != 2:
        raise TypeError("region2d: (H, W) uint8 image")
    h, w = img.shape
    seeds = corner_seeds(h, w) if seeds is None else seeds
    if not img.is_cuda:
        src = img.contiguous()
        reg = torch.empty_like(src)
        arr = (ctypes.c_int * (2 * len(seeds)))(*[c for s in seeds for c in s])
        cpu_lib().pcmx_region2d_serial(src.data_ptr(), w, h, arr, len(seeds), int(threshold), reg.data_ptr())
        return reg
    img_p = pad1(img)
    reg_p = torch.zeros_like(img_p)
    for x, y in seeds:
        if 0 <= x < w and 0 <= y < h:
            reg_p[y + 1, x + 1] = 1
    region2d_grow_padded_(reg_p, img_p, threshold)
    return reg_p[1:-1, 1:-1].contiguous()


def apply_region_mask(img: torch.Tensor, region: torch.Tensor) -> torch.Tensor:
    """image[i] * (region[i] == 0) — the reference's output image (region.c:572-580)."""
    return img * (region == 0).to(img.dtype)


# ------------------------------------------------------------------------------- volumes

SEED_3D = (50, 300, 300)  # (x, y, z), ref raycast.cu:718


def create_volume(dim: int = 512, device="cpu", background: str = "hash", seed: int = 0) -> torch.Tensor:
    """The reference volume (spheres + boxes over a noise background), layout data[z][y][x].

    background="rand": glibc rand()%20 per voxel in z,y,x order — the reference's exact bytes (CPU only).
    background="hash": counter-hash noise, generated on the device (identical on CPU and GPU).
    """
    dev = torch.device(device)
    if background == "rand":
        data = torch.empty(dim, dim, dim, dtype=torch.uint8)
        cpu_lib().pcmx_create_data(data.data_ptr(), dim)
        return data.to(dev)
    if dev.type == "cuda":
        data = torch.empty(dim, dim, dim, dtype=torch.uint8, device=dev)
        return ops().volume_gen_(data, int(seed))
    data = torch.empty(dim, dim, dim, dtype=torch.uint8)
    cpu_lib().pcmx_create_data_hash(data.data_ptr(), dim, int(seed))
    return data


def region3d(data: torch.Tensor, seed=SEED_3D, threshold: int = 1, method: str = "tiled") -> tuple[torch.Tensor, int]:
    """3-D seeded flood fill (6-connected, |a-b| < threshold). Returns (region uint8 0/1, launches)."""
    dim = data.shape[0]
    x, y, z = seed
    if not data.is_cuda:
        reg = torch.empty_like(data)
        cpu_lib().pcmx_region3d_serial(data.contiguous().data_ptr(), dim, x, y, z, int(threshold), reg.data_ptr())
        return reg, 0
    reg = torch.zeros_like(data)
    if method == "naive":
        reg[z, y, x] = 2  # reference frontier semantics (0/1/2)
        n = ops().region3d_grow_(reg, data, int(threshold), False, 1, 1_000_000)
    else:
        reg[z, y, x] = 1
        n = ops().region3d_grow_(reg, data, int(threshold), True, 8, 1_000_000)
    return reg, int(n)


class Camera(ctypes.Structure):
    _fields_ = [("camera", ctypes.c_float * 3), ("forward", ctypes.c_float * 3), ("right", ctypes.c_float * 3),
                ("up", ctypes.c_float * 3), ("pixel_width", ctypes.c_float), ("step_size", ctypes.c_float),
                ("max_steps", ctypes.c_int)]

    def cam12(self) -> list[float]:
        return [*self.camera, *self.forward, *self.right, *self.up]


def default_camera(image_dim: int) -> Camera:
    """Camera of the reference (ref raycast.cu:216-241) computed by the host C code, so the GPU kernels use
    bit-identical constants."""
    cam = Camera()
    lib = cpu_lib()
    lib.pcmx_default_camera.argtypes = [ctypes.c_int, ctypes.POINTER(Camera)]
    lib.pcmx_default_camera(int(image_dim), ctypes.byref(cam))
    return cam


def raycast(data: torch.Tensor, region: torch.Tensor, image_dim: int = 512, method: str = "global",
            cam: Camera | None = None, batch: int = 0, segments: int = 0, variant: int = -1) -> torch.Tensor:
    """Render the volume (ray marching, trilinear sampling of data and region).

    method: "global" — bit-compatible with the reference's serial/global-memory caster (f64 colour update);
            "global_f32" — f32 colour update like the CUDA kernel; "texture" — the texture path
            (texel-centre addressing, correct weights, 8-bit fractional weights) on a packed brick volume;
            `batch` = its march steps per prefetch batch (1, 4, 8, 16: same image; 0 = 16, the fastest);
            `segments` = waves sharing one ray patch, each marching a contiguous share of the steps (1, 2, 4;
            0 = the fastest; partial colours are composed in ray order, so images agree up to f32 rounding);
            `variant` (global methods) = caster variant: -1 the production rule (one ray per 16-lane group up to 2^16
            rays, else the DR16 interleaved volume with one ray per 4-lane group), 0 the round-5 caster (8 steps'
            samples in flight per lane), 1 the one-step-in-flight form, 2 / 3 4 / 16 steps in flight, 4 pair taps,
            5-8 one ray per 64 / 16 / 8 / 4 lanes, 9-11 DR16 layout (lab; identical images).
    """
    cam = cam or default_camera(image_dim)
    if not data.is_cuda:
        if method not in ("global", "serial"):
            raise ValueError("CPU ray casting supports the reference (serial) method only")
        img = torch.empty(image_dim, image_dim, dtype=torch.uint8)
        cpu_lib().pcmx_raycast_serial(data.contiguous().data_ptr(), region.contiguous().data_ptr(), data.shape[0],
                                      image_dim, img.data_ptr())
        return img
    o = ops()
    if method in ("global", "global_f32"):
        return o.raycast_global(data, region, int(image_dim), cam.cam12(), float(cam.pixel_width),
                                float(cam.step_size), int(cam.max_steps), method == "global", int(variant))
    if method == "texture":
        tex = o.brick_pack(data, region)
        return o.raycast_bricked(tex, int(image_dim), cam.cam12(), float(cam.pixel_width), float(cam.step_size),
                                 int(cam.max_steps), int(batch), int(segments))
    raise ValueError(f"unknown raycast method {method!r}")
