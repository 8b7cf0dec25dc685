"""SGEMM (fp32) — ``matrix_multiply`` of ref 1-introduction/matrix.c:63-81 on the MI355X matrix cores.

``sgemm(a, b)`` accepts any shape: tile-aligned problems go straight to the MFMA kernel, others are
zero-padded to the 128x128x32 tile grid first (padding cannot change the product). CPU tensors use the
multithreaded host GEMM of libpcmx_cpu.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import cpu_lib, ops


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def sgemm(a: torch.Tensor, b: torch.Tensor, variant: int = -1) -> torch.Tensor:
    """C = A @ B in fp32 (exact f32 products/sums via v_mfma_f32_32x32x2_f32 on gfx950)."""
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[0]:
        raise ValueError(f"sgemm: incompatible shapes {tuple(a.shape)} x {tuple(b.shape)}")
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise TypeError("sgemm: float32 operands expected")
    m, k = a.shape
    n = b.shape[1]
    if not a.is_cuda:
        ac, bc = a.contiguous(), b.contiguous()
        c = torch.empty(m, n, dtype=torch.float32)
        cpu_lib().pcmx_sgemm_host(ac.data_ptr(), bc.data_ptr(), c.data_ptr(), m, n, k)
        return c
    # pad to the tile of the kernel that will run: 256x256 (K % 64 for the direct-register variant 17 / 18) when the
    # problem fills the chip with 256-tiles (the default dispatch then takes variant 17), else 128x128
    big = variant in (0, 16, 17, 18, 20) or (variant < 0 and -(-m // 256) * -(-n // 256) >= 192)
    tile, kq = (256, 64 if variant in (-1, 17, 18) else 32) if big else (128, 32)  # variant 20: K % 32
    mp, np_, kp = _round_up(m, tile), _round_up(n, tile), _round_up(k, kq)
    ac = a if a.stride(1) == 1 and a.stride(0) % 4 == 0 and a.data_ptr() % 16 == 0 else a.contiguous()
    bc = b if b.stride(1) == 1 and b.stride(0) % 4 == 0 and b.data_ptr() % 16 == 0 else b.contiguous()
    if (mp, np_, kp) == (m, n, k):
        return ops().sgemm(ac, bc, variant)
    ap = F.pad(ac, (0, kp - k, 0, mp - m))
    bp = F.pad(bc, (0, np_ - n, 0, kp - k))
    return ops().sgemm(ap, bp, variant)[:m, :n]


def sgemm_out(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, alpha: float = 1.0, beta: float = 0.0,
              variant: int = -1) -> torch.Tensor:
    """c <- alpha * a @ b + beta * c (tile-aligned GPU operands)."""
    return ops().sgemm_out(a, b, c, float(alpha), float(beta), variant)


def sgemm_simt(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """The CUDA-port-style SIMT kernel (f32 VALU FMAs), kept as the A/B baseline for the MFMA kernel."""
    return ops().sgemm_simt(a, b)


def sgemm_naive_host(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """The reference's i-j-k triple loop (baseline measurement only)."""
    ac, bc = a.contiguous(), b.contiguous()
    c = torch.empty(a.shape[0], b.shape[1], dtype=torch.float32)
    cpu_lib().pcmx_sgemm_naive(ac.data_ptr(), bc.data_ptr(), c.data_ptr(), a.shape[0], b.shape[1], a.shape[1])
    return c
