# round 6: RCCL launch knobs against the SpMV rank step with both exchanges in flight (native path), plus a
# HIP API trace of the same lab to see what RCCL enqueues per exchange (the database stays on the box; only the
# listings come back)
set -o pipefail
mkdir -p gpurun_out/r6/knobs
export SPMV_LAB_N1=0 SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.4
timeout -k 10 240 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/knobs/default.txt 2>&1 && \
NCCL_GRAPH_MIXING_SUPPORT=0 timeout -k 10 240 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/knobs/nomix.txt 2>&1 && \
NCCL_LAUNCH_MODE=GROUP timeout -k 10 240 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/knobs/group.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d /tmp/knobs_trace -o lab -- python3 scripts/spmv_host_lab.py 8 10 > gpurun_out/r6/knobs/trace.txt 2>&1 && \
DB=$(ls /tmp/knobs_trace/*.db /tmp/knobs_trace/*/*.db 2>/dev/null | head -n 1) && echo "db $DB" && ls -la "$DB" && \
python scripts/rocpd_api_window.py "$DB" nccl -5 > gpurun_out/r6/knobs/window_m5.txt && \
python scripts/rocpd_api_window.py "$DB" nccl -6 > gpurun_out/r6/knobs/window_m6.txt && \
python scripts/rocpd_api_window.py "$DB" nccl -40 > gpurun_out/r6/knobs/window_m40.txt
