#!/bin/bash
# One rocprofv3 PMC pass (kernel trace + counters only) over a north-star workload.
# usage: scripts/prof_pmc.sh <outdir> <workload> "<counters>" [--set k=v ...]
out=$1; w=$2; ctr=$3; shift 3
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d "$out" -o p -- \
  python3 -m parallel_c_programs_amd.cli.run_workload "$w" --steps 3 --warmup 1 --no-check "$@" > "$out.log" 2>&1
