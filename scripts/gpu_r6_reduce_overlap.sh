# round 6: the overlapped reduce all-reduce on the GPU box, over gloo with 2 ranks sharing the MI355X (the
# async-work ordering with CUDA tensors; times meaningless), then the same with a perturbed total (must fail)
set -o pipefail
mkdir -p gpurun_out/r6/overlap
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --sections reduce,scan --steps 10 --warmup 3 > gpurun_out/r6/overlap/gloo2.json 2> gpurun_out/r6/overlap/gloo2.err && \
{ timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --sections reduce --steps 5 --warmup 2 --inject-fault reduce:1:perturb > gpurun_out/r6/overlap/gloo2_perturb.json 2> gpurun_out/r6/overlap/gloo2_perturb.err; echo "perturb exit $?" > gpurun_out/r6/overlap/perturb_rc.txt; }
