# round 6: the full-size N = 8 bench path with 8 ranks sharing ONE MI355X over host-staged gloo (times meaningless;
# every check, self-test and the new N > 1 attribution fields are the point)
set -o pipefail
mkdir -p gpurun_out/r6/final
timeout -k 10 1000 python -u bench.py --gpus 8 --backend gloo --steps 10 --warmup 3 > gpurun_out/r6/final/bench_gloo_n8.json 2> gpurun_out/r6/final/bench_gloo_n8.err
