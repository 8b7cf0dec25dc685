"""Torch-facing ops of the MI355X kernels (GPU) with host C fallbacks for CPU tensors."""
from .gemm import sgemm, sgemm_naive_host, sgemm_out, sgemm_simt
from .vector import OP_CODES, axpy_, dot, fill_, rand_uniform_, reduce, scan, vadd, vmul

__all__ = [
    "sgemm", "sgemm_out", "sgemm_simt", "sgemm_naive_host",
    "vmul", "vadd", "axpy_", "dot", "reduce", "scan", "fill_", "rand_uniform_", "OP_CODES",
]
