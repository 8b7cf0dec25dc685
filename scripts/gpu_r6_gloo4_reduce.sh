# round 6: N = 4 gloo (ranks sharing one MI355X), reduce + scan sections only, the overlapped reduce all-reduce
# against the round-5 blocking one (PCMX_REDUCE_OVERLAP=0); stderr is the progress log
set -o pipefail
mkdir -p gpurun_out/r6/gloo4
PCMX_REDUCE_OVERLAP=0 timeout -k 10 400 python -u bench.py --gpus 4 --backend gloo --sections reduce --steps 10 --warmup 3 > gpurun_out/r6/gloo4/ov0.json 2> gpurun_out/r6/gloo4/ov0.err && \
PCMX_REDUCE_OVERLAP=1 timeout -k 10 400 python -u bench.py --gpus 4 --backend gloo --sections reduce --steps 10 --warmup 3 > gpurun_out/r6/gloo4/ov1.json 2> gpurun_out/r6/gloo4/ov1.err && \
timeout -k 10 400 python -u bench.py --gpus 4 --backend gloo --sections scan --steps 10 --warmup 3 > gpurun_out/r6/gloo4/scan.json 2> gpurun_out/r6/gloo4/scan.err
