# round 6: kernel timeline of the N = 8 rank step with the two RCCL self-exchanges (world-1 communicator)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6/prof_spmv_rccl
SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.5 SPMV_LAB_N1=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_spmv_rccl -o run -- python3 scripts/spmv_host_lab.py 8 20 > gpurun_out/r6/prof_spmv_rccl/stdout.txt 2>&1
