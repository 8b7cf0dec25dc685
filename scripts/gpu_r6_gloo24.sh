# round 6: the full-size N = 2 and N = 4 bench paths (the shapes of the driver's scaling runs: slab heights, SpMV
# partitions, chunk bounds) with the ranks sharing ONE MI355X over host-staged gloo; times meaningless, every check,
# self-test and attribution field is the point
set -o pipefail
mkdir -p gpurun_out/r6/gloo24
timeout -k 10 900 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 > gpurun_out/r6/gloo24/bench_gloo_n2.json 2> gpurun_out/r6/gloo24/bench_gloo_n2.err && \
timeout -k 10 900 python -u bench.py --gpus 4 --backend gloo --steps 10 --warmup 3 > gpurun_out/r6/gloo24/bench_gloo_n4.json 2> gpurun_out/r6/gloo24/bench_gloo_n4.err
