# round 6: paired-wave stencil with 5 waves per SIMD forced on the 4-column kernels: N = 8 rank A/B
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 180 --timeout-method thread -k "paired" > gpurun_out/r6/test_stencil_paired2.txt 2>&1 && \
STENCIL_LAB_WORLDS=8,8,8 STENCIL_LAB_DEEP=5 STENCIL_LAB_ONLY=full STENCIL_LAB_PAIRED=0,1 timeout -k 10 300 python -u scripts/stencil_rank_lab.py 6 > gpurun_out/r6/stencil_paired_ab2.txt 2>&1
