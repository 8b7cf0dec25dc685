set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stencil" > gpurun_out/r4l_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/stencil_dma_lab.py 8,6 16384,8192,4096 > gpurun_out/r4l_dma.log 2>&1
