# round 6: the full-size N = 4 bench path, 4 ranks sharing ONE MI355X over host-staged gloo (times meaningless;
# every check, self-test and attribution field is the point). Stacks dumped each 60 s as a heartbeat / hang finder.
set -o pipefail
mkdir -p gpurun_out/r6/gloo4
PCMX_STACK_DUMP_S=60 timeout -k 10 300 python -u bench.py --gpus 4 --backend gloo --sections scan --steps 10 --warmup 3 > gpurun_out/r6/gloo4/scan.json 2> gpurun_out/r6/gloo4/scan.err && \
PCMX_STACK_DUMP_S=60 timeout -k 10 900 python -u bench.py --gpus 4 --backend gloo --steps 10 --warmup 3 > gpurun_out/r6/gloo4/bench_gloo_n4.json 2> gpurun_out/r6/gloo4/bench_gloo_n4.err
