# round 6: full GPU test suite, then the 1-GPU bench line
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/gputest_full.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6/bench_n1.txt 2> gpurun_out/r6/bench_n1.err
