# round 6: N = 8 rank step with the two self-exchanges, torch all_to_all vs the native exchange; + kernel timeline
set -o pipefail
mkdir -p gpurun_out/r6/prof_spmv_native
SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.5 SPMV_LAB_N1=0 timeout -k 10 300 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/spmv_native_f50.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.5 SPMV_LAB_N1=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6/prof_spmv_native -o run -- python3 scripts/spmv_host_lab.py 8 20 > gpurun_out/r6/prof_spmv_native/stdout.txt 2>&1
