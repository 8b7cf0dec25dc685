set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 240 --timeout-method thread -k "rccl_call_shape or probe_failure" > gpurun_out/r6/test_native.txt 2>&1
