set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_apps.py -m gpu -x -q --timeout 120 --timeout-method thread -k "banded or spmv or stencil" > gpurun_out/r4k_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/stencil_dma_lab.py 8,6 16384,8192,4096 > gpurun_out/r4k_dma.log 2>&1 &&
timeout -k 10 200 python -u scripts/spmv_banded_lab.py 100000 401 200 100 200 10 1,8 > gpurun_out/r4k_banded.log 2>&1 &&
timeout -k 10 120 python -u -m parallel_c_programs_amd.cli.run_spmv 100000 401 200 100 200 10 --gpu > gpurun_out/r4k_run_spmv.log 2>&1 &&
STENCIL_LAB_WORLDS=8 STENCIL_LAB_RPW=0,18,24,29,0 timeout -k 10 300 python -u scripts/stencil_rank_lab.py 6 > gpurun_out/r4k_stencil_rank.log 2>&1 &&
timeout -k 10 400 bash scripts/pmc_banded.sh gpurun_out/r4k_banded_pmc > gpurun_out/r4k_banded_pmc.log 2>&1
