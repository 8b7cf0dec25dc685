"""Element-wise, reduction and scan ops.

GPU tensors run the hand-written gfx950 kernels (``torch.ops.pcmx.*``); CPU tensors run the host C library
(OpenMP) or, where the reference has no host routine, an exact torch reference. The CPU path exists so the
distributed algorithms can be exercised with the gloo backend on a GPU-less machine.

Reference parity: vmul = 6-opencl-region-growing/multiply_opencl.cl:1-4 (host check multiply_opencl.c:10-14);
reduce MIN/SUM = the MPI_Allreduce of 2-mpi-region-growing/region.c:437; scan = the histogram CDF
(4-histogram-equalization-openmp-pthreads/histogram_serial.c:29-34) generalised.
"""
from __future__ import annotations

import torch

from .._native import cpu_lib, ops

OP_CODES = {"sum": 0, "min": 1, "max": 2}


def _f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    return t.contiguous()


def vmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """r[i] = a[i] * b[i]."""
    if a.is_cuda:
        return ops().vmul(a, b).view(a.shape)
    a, b = _f32(a, "a"), _f32(b, "b")
    r = torch.empty_like(a)
    cpu_lib().pcmx_vmul_host(a.data_ptr(), b.data_ptr(), r.data_ptr(), a.numel())
    return r


def vadd(a: torch.Tensor, b: torch.Tensor, n_threads: int = 0) -> torch.Tensor:
    """r[i] = a[i] + b[i] (OpenMP on the host, float4 streaming kernel on the GPU)."""
    if a.is_cuda:
        return ops().vadd(a, b).view(a.shape)
    a, b = _f32(a, "a"), _f32(b, "b")
    r = torch.empty_like(a)
    cpu_lib().pcmx_vadd_omp(a.data_ptr(), b.data_ptr(), r.data_ptr(), a.numel(), n_threads)
    return r


def gather_(src: torch.Tensor, idx: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out[i] = src[idx[i]] (int32 indices): the HIP gather kernel on the GPU (the SpMV send-buffer pack),
    torch.index_select on the host. The kernel addresses src with 32-bit byte offsets: a src of 2^29 or more floats
    takes torch.index_select on the GPU too."""
    if src.is_cuda and src.numel() < (1 << 29):
        return ops().gather_(src, idx, out)
    return torch.index_select(src, 0, idx.long(), out=out)


def axpy_(y: torch.Tensor, alpha: float, x: torch.Tensor, n_threads: int = 0) -> torch.Tensor:
    """y <- alpha * x + y in place."""
    if y.is_cuda:
        return ops().axpy_(y, float(alpha), x)
    x = _f32(x, "x")
    assert y.is_contiguous() and y.dtype == torch.float32
    cpu_lib().pcmx_axpy_omp(float(alpha), x.data_ptr(), y.data_ptr(), y.numel(), n_threads)
    return y


def copy_(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """dst <- src (f32): the ticket-ordered streaming kernel on the GPU, torch's copy on the host."""
    if dst.is_cuda:
        return ops().copy_(dst, src)
    return dst.copy_(src)


def dot(a: torch.Tensor, b: torch.Tensor, n_threads: int = 0) -> torch.Tensor:
    """sum(a*b) as a 0-d float32 tensor (f64 host accumulation / f64 final fold on the GPU)."""
    if a.is_cuda:
        return ops().dot(a, b)
    a, b = _f32(a, "a"), _f32(b, "b")
    return torch.tensor(cpu_lib().pcmx_dot_omp(a.data_ptr(), b.data_ptr(), a.numel(), n_threads), dtype=torch.float32)


def reduce(x: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """Global reduction of a float32/int32 tensor to a 0-d tensor (op in sum/min/max)."""
    code = OP_CODES[op]
    if x.is_cuda:
        return ops().reduce(x, code)
    if op == "sum":
        if x.dtype == torch.float32:
            xc = x.contiguous()
            return torch.tensor(cpu_lib().pcmx_sum_omp(xc.data_ptr(), xc.numel(), 0), dtype=torch.float32)
        return x.sum(dtype=torch.int64).to(x.dtype)
    return x.min() if op == "min" else x.max()


def scan(x: torch.Tensor, exclusive: bool = False, init: torch.Tensor | None = None,
         check: bool = False) -> torch.Tensor:
    """Prefix sum over the flattened tensor (decoupled look-back single pass on the GPU).

    ``init`` (a 1-element float32 tensor on the same device) is added to every output; the multi-GPU
    scan feeds its rank offset through it without a host round trip. ``check=True`` waits for the current
    stream and raises if this (or an earlier unchecked) scan on it gave up a look-back (scan_check).
    """
    if x.is_cuda:
        y = ops().scan(x, exclusive, init)
        if check:
            scan_check(x.device)
        return y
    xf = _f32(x, "x").view(-1)
    out = torch.cumsum(xf.double(), 0)
    if exclusive:
        out = torch.cat([out.new_zeros(1), out[:-1]])
    if init is not None:
        out = out + init.double().view(-1)[0]
    return out.float().view(x.shape)


def scan_check(device=None) -> None:
    """Synchronise the current stream of `device` and raise if a scan on it timed out in its look-back."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    ops().scan_check(dev.index if dev.index is not None else torch.cuda.current_device())


def fill_(x: torch.Tensor, value: float) -> torch.Tensor:
    if x.is_cuda:
        return ops().fill_(x, float(value))
    return x.fill_(value)


def rand_uniform_(x: torch.Tensor, seed: int = 0, lo: float = -1.0, hi: float = 1.0) -> torch.Tensor:
    """Counter-based uniform fill generated on the device (no host staging for 1e9-element inputs)."""
    if x.is_cuda:
        return ops().rand_uniform_(x, int(seed), float(lo), float(hi))
    g = torch.Generator().manual_seed(int(seed))
    return x.uniform_(lo, hi, generator=g)
