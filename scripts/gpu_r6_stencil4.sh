# round 6: stencil tests after restricting paired waves to the lab shape
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_multi.py -x -q --timeout 240 --timeout-method thread -k "stencil" > gpurun_out/r6/test_stencil_final.txt 2>&1
