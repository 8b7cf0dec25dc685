# round 6: T = 5 (new instantiation) against T = 6 for one N = 8 / N = 4 rank; bit-exactness first
set -o pipefail
mkdir -p gpurun_out/r6/stencil
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "stencil_fused_steps_bit_exact or stencil_fused_every_lane_geometry" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/stencil/t5_tests.txt 2>&1 && \
STENCIL_LAB_WORLDS=8,4 STENCIL_LAB_DEEP=4,5 STENCIL_LAB_ONLY=full timeout -k 10 300 python -u scripts/stencil_rank_lab.py 6 5 6 5 6 5 > gpurun_out/r6/stencil/t5_t6_rule.txt 2>&1 && \
STENCIL_LAB_WORLDS=8,4 STENCIL_LAB_DEEP=5 STENCIL_LAB_ONLY=full STENCIL_LAB_CPL=4 STENCIL_LAB_RPW=18,24 timeout -k 10 300 python -u scripts/stencil_rank_lab.py 5 6 5 6 > gpurun_out/r6/stencil/t5_t6_cpl4.txt 2>&1
