# round 6: kernel timelines of the T = 5 and T = 6 deep-halo rank steps (why T = 5's deep schedule costs 7% over a
# full launch); the databases stay on the box, the last 30 stencil dispatches (the timed deep5 loop) come back
set -o pipefail
mkdir -p gpurun_out/r6/stencil
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
STENCIL_LAB_WORLDS=8 STENCIL_LAB_DEEP=5 STENCIL_LAB_ONLY=full timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/st5 -o lab -- python3 scripts/stencil_rank_lab.py 5 > gpurun_out/r6/stencil/t5_trace_lab5.txt 2>&1 && \
python scripts/rocpd_timeline.py /tmp/st5/lab_results.db 30 stencil > gpurun_out/r6/stencil/t5_timeline.txt && \
STENCIL_LAB_WORLDS=8 STENCIL_LAB_DEEP=5 STENCIL_LAB_ONLY=full timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/st6 -o lab -- python3 scripts/stencil_rank_lab.py 6 > gpurun_out/r6/stencil/t5_trace_lab6.txt 2>&1 && \
python scripts/rocpd_timeline.py /tmp/st6/lab_results.db 30 stencil > gpurun_out/r6/stencil/t6_timeline.txt
