#!/bin/bash
# Full GPU check of the tree on one MI355X: every GPU test, the driver's bench line, and a rocprofv3 kernel-stats
# profile of a short bench run (summaries go to gpurun_out/<tag>_*; copy the ones to keep into profiles/).
# usage: scripts/gpu_round_check.sh <tag>
set -o pipefail
tag=${1:-check}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 660 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_gputest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o bench -- \
  python3 bench.py --steps 5 --warmup 2 --no-ref > gpurun_out/${tag}_bench_rocprof.log 2>&1
