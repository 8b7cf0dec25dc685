"""Workloads ("models") of the framework: each reference program / north-star config as a step-able object
with a work model (flops, bytes) so every driver reports the same units.

    name          reference ancestor                                   metric
    sgemm         1-introduction/matrix.c:66-79 (matrix_multiply)      TFLOPS (2 n^3)
    reduce        2-mpi-region-growing/region.c:435-440 (Allreduce)    GB/s (4 B/element)
    scan          4-histogram-*/histogram_serial.c:29-34 (CDF)         GB/s (8 B/element)
    stencil       2-mpi-region-growing/region.c:250-353 (halo)         GLUP/s
    spmv          3-serial-optimization/spmv.c:170-177                 GFLOP/s (2 nnz), GB/s
    region2d      2-mpi-region-growing/region.c:493-533                Mpix/s
    region3d      5-cuda-region-growing/raycast.cu:534-822             Mvox/s
    raycast       5-cuda-region-growing/raycast.cu:395-531             Mrays/s
    histeq        4-histogram-*/histogram_serial.c                     Mpix/s
"""
from .workloads import WORKLOADS, build_workload

__all__ = ["WORKLOADS", "build_workload"]
