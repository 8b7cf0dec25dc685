set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_multi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "banded or stencil" > gpurun_out/r4c_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/spmv_banded_lab.py 100000 401 200 100 200 10 1,8 2,3,4,6 > gpurun_out/r4c_banded.log 2>&1 &&
timeout -k 10 400 python -u scripts/stencil_rank_lab.py 6 8 > gpurun_out/r4c_rank.log 2>&1
