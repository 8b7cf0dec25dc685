# round 6: the N = 4 gloo scan section (ranks sharing one MI355X) with every rank's Python stack dumped each 45 s
set -o pipefail
mkdir -p gpurun_out/r6/gloo4
PCMX_STACK_DUMP_S=45 timeout -k 10 300 python -u bench.py --gpus 4 --backend gloo --sections scan --steps 10 --warmup 3 > gpurun_out/r6/gloo4/scan.json 2> gpurun_out/r6/gloo4/scan.err
