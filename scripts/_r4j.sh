set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stencil or banded" > gpurun_out/r4j_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/stencil_rank_lab.py 6 8 > gpurun_out/r4j_stencil_rank.log 2>&1 &&
timeout -k 10 120 python -u -m parallel_c_programs_amd.cli.run_spmv 100000 401 200 100 200 10 --gpu > gpurun_out/r4j_run_spmv.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4j_bench.log 2>&1 &&
timeout -k 10 500 bash scripts/pmc_stencil_bench.sh gpurun_out/r4j_stencil_pmc 8 > gpurun_out/r4j_stencil_pmc.log 2>&1
