# round 6: the N = 8 / N = 4 stencil rank step with its halo exchange on RCCL (world-1 self-exchange, native path)
set -o pipefail
mkdir -p gpurun_out/r6
STENCIL_LAB_RCCL=1 STENCIL_LAB_WORLDS=8,4 STENCIL_LAB_DEEP=5 STENCIL_LAB_ONLY=full,split2 STENCIL_LAB_RPW=0 timeout -k 10 400 python -u scripts/stencil_rank_lab.py 6 6 > gpurun_out/r6/stencil_rccl.txt 2>&1
