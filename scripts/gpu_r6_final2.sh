# round 6, last code state: full GPU tests, smoke, and the 1-GPU bench line
set -o pipefail
mkdir -p gpurun_out/r6/final2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/final2/gputest.txt 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/final2/smoke.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6/final2/bench_line.json 2> gpurun_out/r6/final2/bench.err
