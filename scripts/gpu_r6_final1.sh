# round 6: full GPU tests, the 1-GPU bench line, and the bench under rocprofv3 (kernel stats)
set -o pipefail
mkdir -p gpurun_out/r6/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/final/gputest.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6/final/bench_line.json 2> gpurun_out/r6/final/bench.err && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/final/prof -o bench -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/final/bench_line_under_rocprof.json 2> gpurun_out/r6/final/bench_rocprof.err
