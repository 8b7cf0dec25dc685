set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "banded" > gpurun_out/r4d_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/spmv_banded_lab.py 100000 401 200 100 200 10 1,8 > gpurun_out/r4d_banded.log 2>&1 &&
timeout -k 10 300 bin_lab/stencil_ahead_lab 2048 > gpurun_out/r4d_ahead_2048.log 2>&1 &&
timeout -k 10 300 bin_lab/stencil_ahead_lab 4096 > gpurun_out/r4d_ahead_4096.log 2>&1
