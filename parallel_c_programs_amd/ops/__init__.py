"""Torch-facing ops of the MI355X kernels (GPU) with host C fallbacks for CPU tensors."""
from .gemm import sgemm, sgemm_naive_host, sgemm_out, sgemm_simt
from .halo import pack_edges, unpack_halo_
from .image import (SEED_3D, Camera, apply_region_mask, corner_seeds, create_volume, default_camera, histeq, pad1,
                    raycast, region2d, region2d_grow_padded_, region3d)
from .sparse import CSR, SlicedCSR, banded_csr, create_vector, powerlaw_csr, spmv, spmv_banded
from .stencil import init_grid, stencil5_reference, stencil5_step_, stencil5x2_step_, stencil5_fused_step_, stencil5_fused_spans_
from .vector import OP_CODES, axpy_, copy_, dot, fill_, gather_, rand_uniform_, reduce, scan, scan_check, vadd, vmul

__all__ = [
    "sgemm", "sgemm_out", "sgemm_simt", "sgemm_naive_host",
    "vmul", "vadd", "axpy_", "copy_", "gather_", "dot", "reduce", "scan", "scan_check", "fill_", "rand_uniform_", "OP_CODES",
    "histeq", "region2d", "region2d_grow_padded_", "region3d", "corner_seeds", "pad1", "apply_region_mask",
    "create_volume", "raycast", "default_camera", "Camera", "SEED_3D",
    "stencil5_step_", "stencil5x2_step_", "stencil5_fused_step_", "stencil5_fused_spans_", "stencil5_reference", "init_grid",
    "CSR", "SlicedCSR", "banded_csr", "create_vector", "powerlaw_csr", "spmv", "spmv_banded",
    "pack_edges", "unpack_halo_",
]
