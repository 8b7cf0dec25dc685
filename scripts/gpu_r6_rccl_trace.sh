# round 6: HIP API trace of the SpMV rank lab with both exchanges on the native RCCL path; the database stays on the
# box, only the listings around a few RCCL kernels come back
set -o pipefail
mkdir -p gpurun_out/r6/knobs
export SPMV_LAB_N1=0 SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d /tmp/knobs_trace -o lab -- python3 scripts/spmv_host_lab.py 8 10 > gpurun_out/r6/knobs/trace.txt 2>&1 && \
python scripts/rocpd_api_window.py /tmp/knobs_trace/lab_results.db nccl -5 > gpurun_out/r6/knobs/window_m5.txt && \
python scripts/rocpd_api_window.py /tmp/knobs_trace/lab_results.db nccl -6 > gpurun_out/r6/knobs/window_m6.txt && \
python scripts/rocpd_api_window.py /tmp/knobs_trace/lab_results.db nccl -60 > gpurun_out/r6/knobs/window_m60.txt
