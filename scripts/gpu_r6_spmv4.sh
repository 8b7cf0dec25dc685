# round 6: where the exchange's +30 us per step goes (no-wait / side-stream copy controls) + timeline of the native run
set -o pipefail
mkdir -p gpurun_out/r6/prof_spmv_ctl
SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_N1=0 timeout -k 10 300 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/spmv_controls.txt 2>&1 && \
NCCL_MAX_NCHANNELS=8 SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_N1=0 timeout -k 10 300 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/spmv_controls_nch8.txt 2>&1
