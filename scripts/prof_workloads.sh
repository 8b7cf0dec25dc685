#!/bin/bash
# Kernel-level profile of the north-star workloads (rocprofv3 kernel trace + stats, no counters).
# usage: scripts/prof_workloads.sh <outdir> [workload ...]
set -o pipefail
out=${1:-gpurun_out/prof}; shift
mkdir -p "$out"
ws=${@:-"stencil spmv reduce scan sgemm region3d raycast histeq"}
export TMPDIR=/tmp
for w in $ws; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$w" -o "$w" -- \
    python3 -m parallel_c_programs_amd.cli.run_workload "$w" --steps 10 --warmup 2 --no-check > "$out/$w.log" 2>&1 || exit $?
  tail -n 1 "$out/$w.log"
done
