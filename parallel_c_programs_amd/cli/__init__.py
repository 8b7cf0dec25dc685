"""Command-line entry points with the reference programs' argv and output formats.

    python -m parallel_c_programs_amd.cli.<name> ...      (or torchrun ... -m for the distributed ones)

run_matrix      1-introduction/matrix.c            run_mpi_ring   1-introduction/mpi.c
run_region      2-mpi-region-growing/region.c      run_spmv       3-serial-optimization/spmv.c
run_histogram   4-histogram-equalization-*/        run_raycast    5-cuda-region-growing/raycast.cu,
run_vmul        6-opencl-region-growing/multiply_opencl.c          6-opencl-region-growing/raycast.c
run_device_info print_properties / clutil.c        run_vecops     north-star vector add + dot (CPU/OpenMP)
run_sgemm, run_reduce_scan, run_stencil, run_spmv_dist             north-star GPU configs
"""
