# round 6: T = 6 against T = 8 for one N = 8 / N = 4 rank (2048 / 4096-row slab) with the current kernel and deep
# halo, alternated in one process (auto_fuse picks T = 6 below 6144 rows from round-3 data)
set -o pipefail
mkdir -p gpurun_out/r6/stencil
STENCIL_LAB_WORLDS=8,4 STENCIL_LAB_DEEP=4,5 STENCIL_LAB_ONLY=full timeout -k 10 400 python -u scripts/stencil_rank_lab.py 6 8 6 8 6 8 > gpurun_out/r6/stencil/t6_t8_ab.txt 2>&1
