# round 6 GPU call: raycast variants (DR16) + the SpMV N = 8 rank step with RCCL self-exchanges, chunk 0 at 0.5 / 0.4
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u scripts/raycast_global_lab.py 3 0,4,9,10,11,6,8,0,9,10,11 nogrow > gpurun_out/r6/raycast_lab2.txt 2>&1 && \
SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.5 timeout -k 10 300 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/spmv_rccl_f50.txt 2>&1 && \
SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.4 SPMV_LAB_N1=0 timeout -k 10 300 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/spmv_rccl_f40.txt 2>&1
