# round 6: T = 5 against T = 6 for one N = 8 / N = 4 rank with the deep-halo phases ping-ponging between two buffers
# as StencilSlab does (the lab's earlier one-buffer-per-phase form streams every phase from HBM)
set -o pipefail
mkdir -p gpurun_out/r6/stencil
STENCIL_LAB_WORLDS=8,4 STENCIL_LAB_DEEP=4,5 STENCIL_LAB_ONLY=full timeout -k 10 400 python -u scripts/stencil_rank_lab.py 6 5 6 5 6 5 > gpurun_out/r6/stencil/pingpong_t5_t6.txt 2>&1 && \
STENCIL_LAB_DEEP_BUFS=0 STENCIL_LAB_WORLDS=8 STENCIL_LAB_DEEP=5 STENCIL_LAB_ONLY=full timeout -k 10 300 python -u scripts/stencil_rank_lab.py 6 5 > gpurun_out/r6/stencil/rotating_t5_t6.txt 2>&1
