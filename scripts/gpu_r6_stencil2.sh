# round 6: paired-wave stencil: bit-exactness tests first (bounded), then the rank-lab A/B (paired 0 / 1, 3 passes)
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 240 --timeout-method thread -k "stencil" > gpurun_out/r6/test_stencil_paired.txt 2>&1 && \
STENCIL_LAB_WORLDS=8,4,1 STENCIL_LAB_DEEP=5 STENCIL_LAB_ONLY=full STENCIL_LAB_PAIRED=0,1 timeout -k 10 300 python -u scripts/stencil_rank_lab.py 6 6 6 8 > gpurun_out/r6/stencil_paired_ab.txt 2>&1
