"""pcmx — an MI355X-native (gfx950 / CDNA4) parallel-primitives framework.

Capabilities of anonyomous4/parallel-c-programs, re-designed for MI355X: hand-written HIP kernels
(MFMA/LDS-tiled) exposed as ``torch.ops.pcmx.*``, multi-GPU data parallelism over RCCL/xGMI via
``torch.distributed`` (one process per GPU), and the reference's C entry points / output formats in a
native host library.

Sub-packages
  ops       torch-facing kernels (sgemm, reduce, scan, vmul/vadd/axpy/dot, histogram, stencil, spmv, ...)
  parallel  process groups, Cartesian topology, halo exchange, distributed reduce/scan/stencil/spmv
  models    the reference's applications ("workloads"): region growing 2D/3D, ray casting, SpMV bench,
            histogram equalisation, matrix demo, token ring
  utils     BMP I/O, timers, device info, JSON metrics
  cli       run_* entry points with the reference argv
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401

__all__ = ["__version__"]
