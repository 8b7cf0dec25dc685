# round 6: same-hardware head-to-head with the reference's own OpenCL program (wg256 build, scripts/refbase_build.sh)
# and ours (bin/pipeline3d_opencl: the same program on our HIP kernels), kernel times from rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6/refbase
(cd refbase/wg256 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6/refbase/ref" -o ref -- ./raycast_timed > "$R/gpurun_out/r6/refbase/ref_stdout.txt" 2>&1) && \
(cd gpurun_out/r6/refbase && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6/refbase/ours" -o ours -- "$R/bin/pipeline3d_opencl" > "$R/gpurun_out/r6/refbase/ours_stdout.txt" 2>&1)
