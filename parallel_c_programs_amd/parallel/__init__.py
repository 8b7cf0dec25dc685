"""Distribution layer: one process per MI355X over RCCL/xGMI (gloo on CPU for tests).

Replaces the reference's MPI programs (1-introduction/mpi.c, 2-mpi-region-growing/region.c).
"""
from .collectives import allreduce_buckets, gather_rows, global_reduce, global_scan, scatter_rows
from .dist import Context, LazyContext, finalize, free_port, init, spawn
from .halo import HaloExchanger2D
from .region2d import gather_tiles, grow_distributed, scatter_tiles
from .ring import token_ring
from .spmv import DistributedSpMV, nnz_balanced_cuts
from .stencil import StencilSlab, auto_fuse, auto_halo_mult, reference_run
from .topology import CartTopology, dims_create, prime_factors, split
from .volume3d import DistributedVolume, VolumeSlab, emulate_slabs

__all__ = [
    "LazyContext",
    "Context", "init", "finalize", "spawn", "free_port",
    "CartTopology", "dims_create", "prime_factors", "split",
    "HaloExchanger2D", "global_reduce", "global_scan", "allreduce_buckets", "scatter_rows", "gather_rows",
    "grow_distributed", "scatter_tiles", "gather_tiles", "token_ring",
    "DistributedSpMV", "nnz_balanced_cuts", "StencilSlab", "auto_fuse", "auto_halo_mult", "reference_run",
    "DistributedVolume", "VolumeSlab", "emulate_slabs",
]
