# round 6: chunk 0 at 0.4 of the rows, native exchange: step times and the kernel timeline
set -o pipefail
mkdir -p gpurun_out/r6/prof_spmv_native_f40
SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.4 SPMV_LAB_N1=0 timeout -k 10 300 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/spmv_native_f40.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.4 SPMV_LAB_N1=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6/prof_spmv_native_f40 -o run -- python3 scripts/spmv_host_lab.py 8 20 > gpurun_out/r6/prof_spmv_native_f40/stdout.txt 2>&1
