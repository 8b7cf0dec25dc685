set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_gpu_core.py -x -q --timeout 120 --timeout-method thread -k "vmul or ticket or fill or copy or axpy" > gpurun_out/r6/test_vec.txt 2>&1 && \
timeout -k 10 200 python -u scripts/kbench.py --what vec --reps 10 > gpurun_out/r6/kbench_vec.txt 2>&1
